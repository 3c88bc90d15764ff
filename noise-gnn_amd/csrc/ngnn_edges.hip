// Edge validation and COO -> CSR grouping (stable) for the aggregation path.
//
// Replaces the index handling PyG 2.5.1 does implicitly inside
// MessagePassing.propagate (index_select by edge_index[0], scatter by
// edge_index[1]) for the reference's conv calls at
// src/models/layers/sage.py:34 and src/models/layers/convolution.py:31.
//
// Design (MI355X): NeighborLoader blocks arrive target-sorted
// (pipeline.py:152-155), so the common path is two embarrassingly parallel,
// HBM-streaming kernels (int64 -> int32 narrowing copy + a lower_bound per
// row).  Unsorted inputs (rewired edges, augmentation.py:82-85, are
// source-sorted) take a stable LSD radix sort limited to ceil(log2 n_rows)
// key bits.  Stability keeps edge order inside each row, so every per-row
// reduction downstream runs in PyG's CPU scatter order.
#include <hipcub/hipcub.hpp>

#include "ngnn_internal.h"

namespace ngnn {
namespace {

__global__ __launch_bounds__(256) void k_edge_probe(const int64_t *__restrict__ src,
                                                    const int64_t *__restrict__ dst, int64_t E,
                                                    int64_t n_src, int64_t n_dst,
                                                    int32_t *__restrict__ status) {
    int bad_s = 0, bad_d = 0, uns_d = 0, uns_s = 0;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = src[e], d = dst[e];
        bad_s |= (s < 0) | (s >= n_src);
        bad_d |= (d < 0) | (d >= n_dst);
        if (e > 0) {
            uns_d |= dst[e - 1] > d;
            uns_s |= src[e - 1] > s;
        }
    }
    // block-level OR, then at most one atomic per block and flag (grid <= 256 blocks)
    const int flags = bad_s | (bad_d << 1) | (uns_d << 2) | (uns_s << 3);
    const int any = __syncthreads_or(flags != 0);
    if (!any) return;
    __shared__ int acc;
    if (threadIdx.x == 0) acc = 0;
    __syncthreads();
    if (flags) atomicOr(&acc, flags);
    __syncthreads();
    if (threadIdx.x == 0) {
        const int f = acc;
        if (f & 1) atomicOr(status + 0, 1);
        if (f & 2) atomicOr(status + 1, 1);
        if (f & 4) atomicOr(status + 2, 1);
        if (f & 8) atomicOr(status + 3, 1);
    }
}

// rowptr[i] = first position p with keys[p] >= i   (i in [0, n_rows])
template <typename K>
__global__ __launch_bounds__(256) void k_rowptr_lower_bound(const K *__restrict__ keys, int32_t E,
                                                            int32_t n_rows,
                                                            int32_t *__restrict__ rowptr) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i > n_rows) return;
    int32_t lo = 0, hi = E;
    while (lo < hi) {
        const int32_t mid = lo + ((hi - lo) >> 1);
        if ((int64_t)keys[mid] < i)
            lo = mid + 1;
        else
            hi = mid;
    }
    rowptr[i] = lo;
}

__global__ __launch_bounds__(256) void k_narrow_copy(const int64_t *__restrict__ vals, int32_t E,
                                                     int32_t *__restrict__ col,
                                                     int32_t *__restrict__ eid) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
         e += (int64_t)gridDim.x * blockDim.x) {
        col[e] = static_cast<int32_t>(vals[e]);
        if (eid) eid[e] = static_cast<int32_t>(e);
    }
}

__global__ __launch_bounds__(256) void k_keys_iota(const int64_t *__restrict__ keys, int32_t E,
                                                   int32_t *__restrict__ k32,
                                                   int32_t *__restrict__ iota) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
         e += (int64_t)gridDim.x * blockDim.x) {
        k32[e] = static_cast<int32_t>(keys[e]);
        iota[e] = static_cast<int32_t>(e);
    }
}

__global__ __launch_bounds__(256) void k_permute_vals(const int64_t *__restrict__ vals,
                                                      const int32_t *__restrict__ perm, int32_t E,
                                                      int32_t *__restrict__ col,
                                                      int32_t *__restrict__ eid) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < E;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int32_t p = perm[k];
        col[k] = static_cast<int32_t>(vals[p]);
        if (eid) eid[k] = p;
    }
}

inline int key_bits(int64_t n_rows) {
    int b = 1;
    while (b < 31 && (int64_t(1) << b) < n_rows) ++b;
    return b;
}

inline unsigned stream_grid(int64_t n, int block = 256, int64_t cap = 256 * 16) {
    int64_t g = ceil_div(n > 0 ? n : 1, block);
    return static_cast<unsigned>(g < cap ? g : cap);
}

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

size_t cub_temp_bytes(int64_t E, int64_t n_rows) {
    size_t temp = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, temp, (const int32_t *)nullptr, (int32_t *)nullptr,
                                       (const int32_t *)nullptr, (int32_t *)nullptr,
                                       static_cast<int>(E), 0, key_bits(n_rows));
    return temp;
}

}  // namespace
}  // namespace ngnn

using namespace ngnn;

extern "C" int ngnn_edge_probe(const int64_t *edge_index, int64_t E, int64_t n_src, int64_t n_dst,
                               int32_t *status, void *stream) {
    NGNN_RETURN_IF(!status || E < 0 || n_src < 0 || n_dst < 0, NGNN_E_ARG);
    NGNN_RETURN_IF(E > 0 && !edge_index, NGNN_E_ARG);
    NGNN_RETURN_IF(!fits_i32(E) || !fits_i32(n_src) || !fits_i32(n_dst), NGNN_E_RANGE);
    if (E == 0) return NGNN_OK;
    hipLaunchKernelGGL(k_edge_probe, dim3(stream_grid(E, 256, 256)), dim3(256), 0, as_stream(stream),
                       edge_index, edge_index + E, E, n_src, n_dst, status);
    return launch_status();
}

extern "C" size_t ngnn_csr_workspace_bytes(int64_t E, int64_t n_rows) {
    if (E <= 0) return 0;
    return 4 * align_up(sizeof(int32_t) * (size_t)E, 256) + align_up(cub_temp_bytes(E, n_rows), 256);
}

extern "C" int ngnn_csr_build(const int64_t *keys, const int64_t *vals, int64_t E, int64_t n_rows,
                              int keys_sorted, int32_t *rowptr, int32_t *col, int32_t *eid,
                              void *ws, size_t ws_bytes, void *stream) {
    NGNN_RETURN_IF(E < 0 || n_rows < 0 || !rowptr, NGNN_E_ARG);
    NGNN_RETURN_IF(E > 0 && (!keys || !vals || !col), NGNN_E_ARG);
    NGNN_RETURN_IF(!fits_i32(E) || !fits_i32(n_rows + 1), NGNN_E_RANGE);
    hipStream_t st = as_stream(stream);
    const int32_t E32 = static_cast<int32_t>(E), R32 = static_cast<int32_t>(n_rows);
    const unsigned grid_rows = static_cast<unsigned>(ceil_div(n_rows + 1, 256));
    if (E == 0) {
        hipLaunchKernelGGL(k_rowptr_lower_bound<int64_t>, dim3(grid_rows), dim3(256), 0, st,
                           keys, 0, R32, rowptr);
        return launch_status();
    }
    if (keys_sorted) {
        hipLaunchKernelGGL(k_narrow_copy, dim3(stream_grid(E)), dim3(256), 0, st, vals, E32, col,
                           eid);
        hipLaunchKernelGGL(k_rowptr_lower_bound<int64_t>, dim3(grid_rows), dim3(256), 0, st, keys,
                           E32, R32, rowptr);
        return launch_status();
    }
    const size_t need = ngnn_csr_workspace_bytes(E, n_rows);
    NGNN_RETURN_IF(!ws || ws_bytes < need, NGNN_E_WORKSPACE);
    char *p = static_cast<char *>(ws);
    const size_t slab = align_up(sizeof(int32_t) * (size_t)E, 256);
    int32_t *k_in = reinterpret_cast<int32_t *>(p);
    int32_t *k_out = reinterpret_cast<int32_t *>(p + slab);
    int32_t *v_in = reinterpret_cast<int32_t *>(p + 2 * slab);
    int32_t *v_out = reinterpret_cast<int32_t *>(p + 3 * slab);
    void *temp = p + 4 * slab;
    size_t temp_bytes = need - 4 * slab;
    hipLaunchKernelGGL(k_keys_iota, dim3(stream_grid(E)), dim3(256), 0, st, keys, E32, k_in, v_in);
    hipError_t err = hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, k_in, k_out, v_in, v_out,
                                                        E32, 0, key_bits(n_rows), st);
    if (err != hipSuccess) return static_cast<int>(err);
    hipLaunchKernelGGL(k_permute_vals, dim3(stream_grid(E)), dim3(256), 0, st, vals, v_out, E32,
                       col, eid);
    hipLaunchKernelGGL(k_rowptr_lower_bound<int32_t>, dim3(grid_rows), dim3(256), 0, st, k_out,
                       E32, R32, rowptr);
    return launch_status();
}
