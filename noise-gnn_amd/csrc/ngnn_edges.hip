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
// key bits: in-tree counting passes over 4-bit digits (per pass: per-block
// digit counts, one exclusive scan of the [digit][block] counts, a stable
// scatter in which every thread places its 16 consecutive items in order).
// Stability keeps edge order inside each row, so every per-row reduction
// downstream runs in PyG's CPU scatter order.

#include <utility>

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

// ---- stable LSD radix sort of (key, value) int32 pairs, 4-bit digits
constexpr int RS_T = 256;           // threads per block
constexpr int RS_IPT = 16;          // consecutive items per thread
constexpr int RS_CH = RS_T * RS_IPT;  // items per block
constexpr int RS_D = 16;            // digits

// hist[d * nb + b] = #{items of block b with digit d}
__global__ __launch_bounds__(RS_T) void k_rs_hist(const int32_t *__restrict__ keys, int32_t E, int shift,
                                                  int32_t *__restrict__ hist) {
    __shared__ int cnt[RS_D][RS_T + 1];
    const int t = threadIdx.x, b = blockIdx.x, nb = gridDim.x;
#pragma unroll
    for (int d = 0; d < RS_D; ++d) cnt[d][t] = 0;
    const int64_t i0 = static_cast<int64_t>(b) * RS_CH + static_cast<int64_t>(t) * RS_IPT;
    for (int i = 0; i < RS_IPT; ++i)
        if (i0 + i < E) ++cnt[(keys[i0 + i] >> shift) & (RS_D - 1)][t];
    __syncthreads();
    if (t < RS_D) {
        int s = 0;
        for (int j = 0; j < RS_T; ++j) s += cnt[t][j];
        hist[t * nb + b] = s;
    }
}

// in place exclusive scan of n ints (one block of 1024 threads, chunks of 1024)
__global__ __launch_bounds__(1024) void k_rs_scan(int32_t *__restrict__ v, int n) {
    __shared__ int s[1024];
    __shared__ int carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int c0 = 0; c0 < n; c0 += 1024) {
        const int i = c0 + threadIdx.x;
        const int x = i < n ? v[i] : 0;
        s[threadIdx.x] = x;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele
            const int y = threadIdx.x >= o ? s[threadIdx.x - o] : 0;
            __syncthreads();
            s[threadIdx.x] += y;
            __syncthreads();
        }
        const int base = carry;
        if (i < n) v[i] = base + s[threadIdx.x] - x;
        __syncthreads();
        if (threadIdx.x == 1023) carry = base + s[1023];
        __syncthreads();
    }
}

// stable scatter: item order is block, then thread, then the thread's own
// items in sequence -- the input order
__global__ __launch_bounds__(RS_T) void k_rs_scatter(const int32_t *__restrict__ kin, const int32_t *__restrict__ vin,
                                                     int32_t E, int shift, const int32_t *__restrict__ off,
                                                     int32_t *__restrict__ kout, int32_t *__restrict__ vout) {
    __shared__ int cnt[RS_D][RS_T + 1];
    const int t = threadIdx.x, b = blockIdx.x, nb = gridDim.x;
#pragma unroll
    for (int d = 0; d < RS_D; ++d) cnt[d][t] = 0;
    const int64_t i0 = static_cast<int64_t>(b) * RS_CH + static_cast<int64_t>(t) * RS_IPT;
    int k[RS_IPT], v[RS_IPT];
#pragma unroll
    for (int i = 0; i < RS_IPT; ++i) {
        const bool ok = i0 + i < E;
        k[i] = ok ? kin[i0 + i] : 0;
        v[i] = ok ? vin[i0 + i] : 0;
        if (ok) ++cnt[(k[i] >> shift) & (RS_D - 1)][t];
    }
    __syncthreads();
    // exclusive scan of every digit row over the threads (Hillis-Steele)
    for (int o = 1; o < RS_T; o <<= 1) {
        int y[RS_D];
#pragma unroll
        for (int d = 0; d < RS_D; ++d) y[d] = t >= o ? cnt[d][t - o] : 0;
        __syncthreads();
#pragma unroll
        for (int d = 0; d < RS_D; ++d) cnt[d][t] += y[d];
        __syncthreads();
    }
    // cnt[d][t] is now inclusive: this thread's first slot per digit
    int base[RS_D];
#pragma unroll
    for (int d = 0; d < RS_D; ++d) base[d] = off[d * nb + b] + (t > 0 ? cnt[d][t - 1] : 0);
    __syncthreads();
#pragma unroll
    for (int d = 0; d < RS_D; ++d) cnt[d][t] = base[d];  // running positions, one slot per thread
#pragma unroll
    for (int i = 0; i < RS_IPT; ++i) {
        if (i0 + i < E) {
            const int d = (k[i] >> shift) & (RS_D - 1);
            const int pos = cnt[d][t]++;
            kout[pos] = k[i];
            vout[pos] = v[i];
        }
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

// the [digit][block] counts of one pass
size_t rs_temp_bytes(int64_t E) { return sizeof(int32_t) * RS_D * static_cast<size_t>(ceil_div(E, RS_CH)); }

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
    (void)n_rows;
    return 4 * align_up(sizeof(int32_t) * (size_t)E, 256) + align_up(rs_temp_bytes(E), 256);
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
    (void)temp_bytes;
    hipLaunchKernelGGL(k_keys_iota, dim3(stream_grid(E)), dim3(256), 0, st, keys, E32, k_in, v_in);
    const int nb = static_cast<int>(ceil_div(E, RS_CH));
    int32_t *hist = static_cast<int32_t *>(temp);
    const int bits = key_bits(n_rows);
    for (int shift = 0; shift < bits; shift += 4) {  // (ping-pong: the result of each pass in k_out, v_out)
        hipLaunchKernelGGL(k_rs_hist, dim3(nb), dim3(RS_T), 0, st, k_in, E32, shift, hist);
        hipLaunchKernelGGL(k_rs_scan, dim3(1), dim3(1024), 0, st, hist, RS_D * nb);
        hipLaunchKernelGGL(k_rs_scatter, dim3(nb), dim3(RS_T), 0, st, k_in, v_in, E32, shift, hist, k_out, v_out);
        std::swap(k_in, k_out);
        std::swap(v_in, v_out);
    }
    // (the sorted pairs are in k_in / v_in after the last swap)
    hipLaunchKernelGGL(k_permute_vals, dim3(stream_grid(E)), dim3(256), 0, st, vals, v_in, E32,
                       col, eid);
    hipLaunchKernelGGL(k_rowptr_lower_bound<int32_t>, dim3(grid_rows), dim3(256), 0, st, k_in,
                       E32, R32, rowptr);
    return launch_status();
}
