// Segment (per-target-row) aggregation over a CSR neighbour block, fp32.
//
// Replaces PyG 2.5.1 MessagePassing.propagate for a Tensor edge_index
// (x.index_select(0, src) materialising [E,F] messages, then
// zeros.scatter_add_ / scatter_reduce_ by target) as used by SAGEConv
// (sage.py:34) and GCNConv (convolution.py:31).  No [E,F] message tensor
// and no atomics: one group of LPR lanes owns one target row, walks its
// neighbour list in edge order and keeps the running reduction in registers,
// so fp32 results are bit-identical to the CPU scatter order.
//
// Layout / MI355X mapping
//   * rows are gathered whole: VEC-wide (16 B for VEC=4) coalesced loads,
//     LPR = next_pow2(F/VEC) lanes per row (F=100 -> 25 of 32 lanes, F=256
//     -> one wave per row), 256-thread blocks = 256/LPR rows per block.
//   * neighbour ids are loaded once per group (lane k loads col[beg+k]) and
//     broadcast with __shfl (ds_bpermute) instead of LPR redundant loads.
//   * four neighbour rows are in flight per lane before they are reduced in
//     order (memory-level parallelism without reordering the fp32 sum).
//   * HBM-bound: bytes per row = deg*(F*4 + 4) + 8 + F*4.
#include "ngnn_internal.h"

namespace ngnn {
namespace {

template <int VEC>
struct Vec;
template <>
struct Vec<4> {
    using T = float4;
};
template <>
struct Vec<2> {
    using T = float2;
};
template <>
struct Vec<1> {
    using T = float;
};

template <int VEC>
__device__ __forceinline__ float &comp(typename Vec<VEC>::T &v, int i) {
    return reinterpret_cast<float *>(&v)[i];
}

template <int VEC>
__device__ __forceinline__ float comp(const typename Vec<VEC>::T &v, int i) {
    return reinterpret_cast<const float *>(&v)[i];
}

template <int VEC>
__device__ __forceinline__ typename Vec<VEC>::T splat(float s) {
    typename Vec<VEC>::T v;
#pragma unroll
    for (int i = 0; i < VEC; ++i) comp<VEC>(v, i) = s;
    return v;
}

template <int VEC>
__device__ __forceinline__ typename Vec<VEC>::T ld(const float *p) {
    return *reinterpret_cast<const typename Vec<VEC>::T *>(p);
}

template <int VEC>
__device__ __forceinline__ void st(float *p, const typename Vec<VEC>::T &v) {
    *reinterpret_cast<typename Vec<VEC>::T *>(p) = v;
}

// torch amax semantics: NaN propagates, otherwise the larger value wins.
__device__ __forceinline__ float nanmax(float acc, float v) {
    return (acc != acc) ? acc : ((v != v || v > acc) ? v : acc);
}

template <int VEC, int RED>
__device__ __forceinline__ void reduce_into(typename Vec<VEC>::T &acc,
                                            const typename Vec<VEC>::T &v) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
        float &a = comp<VEC>(acc, i);
        const float b = reinterpret_cast<const float *>(&v)[i];
        a = (RED == NGNN_REDUCE_MAX) ? nanmax(a, b) : a + b;
    }
}

// --------------------------------------------------------------- forward
template <int VEC, int LPR, int RED>
__global__ __launch_bounds__(256) void k_seg_agg_fwd(const float *__restrict__ x, int64_t ldx,
                                                     int F, const int32_t *__restrict__ rowptr,
                                                     const int32_t *__restrict__ col, int n_dst,
                                                     float *__restrict__ out, int64_t ldo) {
    using V = typename Vec<VEC>::T;
    constexpr int GROUPS = 256 / LPR;
    constexpr int UNR = 4;
    const int lane = threadIdx.x % LPR;
    const int64_t row = (int64_t)blockIdx.x * GROUPS + threadIdx.x / LPR;
    if (row >= n_dst) return;  // whole group leaves together
    const int beg = rowptr[row], end = rowptr[row + 1];
    const int nchunks = (F + LPR * VEC - 1) / (LPR * VEC);
    for (int ch = 0; ch < nchunks; ++ch) {
        const int f = ch * LPR * VEC + lane * VEC;
        const bool act = f < F;
        V acc = splat<VEC>(RED == NGNN_REDUCE_MAX ? -INFINITY : 0.0f);
        for (int eb = beg; eb < end; eb += LPR) {
            const int n = min(LPR, end - eb);
            const int myc = lane < n ? col[eb + lane] : 0;
            int k = 0;
            for (; k + UNR <= n; k += UNR) {
                int c[UNR];
                V v[UNR];
#pragma unroll
                for (int u = 0; u < UNR; ++u) c[u] = __shfl(myc, k + u, LPR);
                if (act) {
#pragma unroll
                    for (int u = 0; u < UNR; ++u) v[u] = ld<VEC>(x + (int64_t)c[u] * ldx + f);
#pragma unroll
                    for (int u = 0; u < UNR; ++u) reduce_into<VEC, RED>(acc, v[u]);
                }
            }
            for (; k < n; ++k) {
                const int c0 = __shfl(myc, k, LPR);
                if (act) reduce_into<VEC, RED>(acc, ld<VEC>(x + (int64_t)c0 * ldx + f));
            }
        }
        if (!act) continue;
        const int deg = end - beg;
        if (RED == NGNN_REDUCE_MEAN) {
            const float cnt = static_cast<float>(deg > 1 ? deg : 1);
#pragma unroll
            for (int i = 0; i < VEC; ++i) comp<VEC>(acc, i) = comp<VEC>(acc, i) / cnt;
        } else if (RED == NGNN_REDUCE_MAX && deg == 0) {
            acc = splat<VEC>(0.0f);
        }
        st<VEC>(out + row * ldo + f, acc);
    }
}

// bf16 input rows (a bf16 model's activations): one wave per target row,
// lanes over 4-column quads (8-B loads), widened exactly and reduced in edge
// order in fp32 -- the sequence of the fp32 kernel on the widened rows.
template <int RED>
__global__ __launch_bounds__(256) void k_seg_agg_fwd_bf16(const uint16_t *__restrict__ x, int64_t ldx,
                                                          int F, const int32_t *__restrict__ rowptr,
                                                          const int32_t *__restrict__ col, int n_dst,
                                                          float *__restrict__ out, int64_t ldo) {
    const int lane = threadIdx.x & 63;
    const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (row >= n_dst) return;
    const int beg = rowptr[row], end = rowptr[row + 1];
    for (int f = 4 * lane; f < F; f += 256) {
        float4 acc = splat<4>(RED == NGNN_REDUCE_MAX ? -INFINITY : 0.0f);
        for (int e = beg; e < end; ++e) {
            const int64_t j = col[e];
            const uint2 w = *reinterpret_cast<const uint2 *>(x + j * ldx + f);
            const float4 v{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                           __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u)};
            reduce_into<4, RED>(acc, v);
        }
        const int deg = end - beg;
        if (RED == NGNN_REDUCE_MEAN) {
            const float cnt = static_cast<float>(deg > 1 ? deg : 1);
#pragma unroll
            for (int i = 0; i < 4; ++i) comp<4>(acc, i) = comp<4>(acc, i) / cnt;
        } else if (RED == NGNN_REDUCE_MAX && deg == 0) {
            acc = splat<4>(0.0f);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (f + i < F) out[row * ldo + f + i] = comp<4>(acc, i);
    }
}

// ------------------------------------------------- backward, sum / mean
// grad_x[j] = sum_{e: src_e = j} g[dst_e] (/ deg(dst_e) for mean), over the
// transposed CSR (rowptr_t, col_t = targets) in edge order.
template <int VEC, int LPR, int RED>
__global__ __launch_bounds__(256) void k_seg_agg_bwd_sum(
    const float *__restrict__ g, int64_t ldg, int F, const int32_t *__restrict__ rowptr,
    const int32_t *__restrict__ rowptr_t, const int32_t *__restrict__ col_t, int n_src,
    float *__restrict__ gx, int64_t ldgx) {
    using V = typename Vec<VEC>::T;
    constexpr int GROUPS = 256 / LPR;
    constexpr int UNR = 4;
    const int lane = threadIdx.x % LPR;
    const int64_t row = (int64_t)blockIdx.x * GROUPS + threadIdx.x / LPR;
    if (row >= n_src) return;
    const int beg = rowptr_t[row], end = rowptr_t[row + 1];
    const int nchunks = (F + LPR * VEC - 1) / (LPR * VEC);
    for (int ch = 0; ch < nchunks; ++ch) {
        const int f = ch * LPR * VEC + lane * VEC;
        const bool act = f < F;
        V acc = splat<VEC>(0.0f);
        for (int eb = beg; eb < end; eb += LPR) {
            const int n = min(LPR, end - eb);
            int myd = 0;
            float mycnt = 1.0f;
            if (lane < n) {
                myd = col_t[eb + lane];
                if (RED == NGNN_REDUCE_MEAN) {
                    const int dg = rowptr[myd + 1] - rowptr[myd];
                    mycnt = static_cast<float>(dg > 1 ? dg : 1);
                }
            }
            int k = 0;
            for (; k + UNR <= n; k += UNR) {
                int d[UNR];
                float cn[UNR];
                V v[UNR];
#pragma unroll
                for (int u = 0; u < UNR; ++u) {
                    d[u] = __shfl(myd, k + u, LPR);
                    cn[u] = __shfl(mycnt, k + u, LPR);
                }
                if (act) {
#pragma unroll
                    for (int u = 0; u < UNR; ++u) v[u] = ld<VEC>(g + (int64_t)d[u] * ldg + f);
#pragma unroll
                    for (int u = 0; u < UNR; ++u) {
#pragma unroll
                        for (int i = 0; i < VEC; ++i) {
                            const float t = comp<VEC>(v[u], i);
                            comp<VEC>(acc, i) += (RED == NGNN_REDUCE_MEAN) ? t / cn[u] : t;
                        }
                    }
                }
            }
            for (; k < n; ++k) {
                const int d0 = __shfl(myd, k, LPR);
                const float c0 = __shfl(mycnt, k, LPR);
                if (act) {
                    V v0 = ld<VEC>(g + (int64_t)d0 * ldg + f);
#pragma unroll
                    for (int i = 0; i < VEC; ++i) {
                        const float t = comp<VEC>(v0, i);
                        comp<VEC>(acc, i) += (RED == NGNN_REDUCE_MEAN) ? t / c0 : t;
                    }
                }
            }
        }
        if (act) st<VEC>(gx + row * ldgx + f, acc);
    }
}

// ------------------------------------------------------ backward, max
// Pass A (forward CSR): gdist[i,f] = g[i,f] / ([agg==0] + #{e: x[src_e,f]==agg[i,f]})
template <int VEC, int LPR>
__global__ __launch_bounds__(256) void k_max_bwd_dist(
    const float *__restrict__ g, int64_t ldg, int F, const int32_t *__restrict__ rowptr,
    const int32_t *__restrict__ col, int n_dst, const float *__restrict__ x, int64_t ldx,
    const float *__restrict__ agg, int64_t lda, float *__restrict__ gdist) {
    using V = typename Vec<VEC>::T;
    constexpr int GROUPS = 256 / LPR;
    const int lane = threadIdx.x % LPR;
    const int64_t row = (int64_t)blockIdx.x * GROUPS + threadIdx.x / LPR;
    if (row >= n_dst) return;
    const int beg = rowptr[row], end = rowptr[row + 1];
    const int nchunks = (F + LPR * VEC - 1) / (LPR * VEC);
    for (int ch = 0; ch < nchunks; ++ch) {
        const int f = ch * LPR * VEC + lane * VEC;
        const bool act = f < F;
        V a = act ? ld<VEC>(agg + row * lda + f) : splat<VEC>(0.0f);
        V ties;
#pragma unroll
        for (int i = 0; i < VEC; ++i) comp<VEC>(ties, i) = comp<VEC>(a, i) == 0.0f ? 1.0f : 0.0f;
        for (int eb = beg; eb < end; eb += LPR) {
            const int n = min(LPR, end - eb);
            const int myc = lane < n ? col[eb + lane] : 0;
            for (int k = 0; k < n; ++k) {
                const int c0 = __shfl(myc, k, LPR);
                if (act) {
                    V v = ld<VEC>(x + (int64_t)c0 * ldx + f);
#pragma unroll
                    for (int i = 0; i < VEC; ++i)
                        comp<VEC>(ties, i) += (comp<VEC>(v, i) == comp<VEC>(a, i)) ? 1.0f : 0.0f;
                }
            }
        }
        if (!act) continue;
        V gv = ld<VEC>(g + row * ldg + f);
#pragma unroll
        for (int i = 0; i < VEC; ++i) comp<VEC>(gv, i) = comp<VEC>(gv, i) / comp<VEC>(ties, i);
        st<VEC>(gdist + row * (int64_t)F + f, gv);
    }
}

// Pass B (transposed CSR): grad_x[j,f] = sum_e [x[j,f]==agg[d_e,f]] * gdist[d_e,f]
template <int VEC, int LPR>
__global__ __launch_bounds__(256) void k_max_bwd_gather(
    const float *__restrict__ gdist, int F, const int32_t *__restrict__ rowptr_t,
    const int32_t *__restrict__ col_t, int n_src, const float *__restrict__ x, int64_t ldx,
    const float *__restrict__ agg, int64_t lda, float *__restrict__ gx, int64_t ldgx) {
    using V = typename Vec<VEC>::T;
    constexpr int GROUPS = 256 / LPR;
    const int lane = threadIdx.x % LPR;
    const int64_t row = (int64_t)blockIdx.x * GROUPS + threadIdx.x / LPR;
    if (row >= n_src) return;
    const int beg = rowptr_t[row], end = rowptr_t[row + 1];
    const int nchunks = (F + LPR * VEC - 1) / (LPR * VEC);
    for (int ch = 0; ch < nchunks; ++ch) {
        const int f = ch * LPR * VEC + lane * VEC;
        const bool act = f < F;
        const V xv = act ? ld<VEC>(x + row * ldx + f) : splat<VEC>(0.0f);
        V acc = splat<VEC>(0.0f);
        for (int eb = beg; eb < end; eb += LPR) {
            const int n = min(LPR, end - eb);
            const int myd = lane < n ? col_t[eb + lane] : 0;
            for (int k = 0; k < n; ++k) {
                const int d0 = __shfl(myd, k, LPR);
                if (act) {
                    const V av = ld<VEC>(agg + (int64_t)d0 * lda + f);
                    const V gd = ld<VEC>(gdist + (int64_t)d0 * F + f);
#pragma unroll
                    for (int i = 0; i < VEC; ++i) {
                        const float m = (comp<VEC>(xv, i) == reinterpret_cast<const float *>(&av)[i])
                                            ? 1.0f
                                            : 0.0f;
                        comp<VEC>(acc, i) += m * reinterpret_cast<const float *>(&gd)[i];
                    }
                }
            }
        }
        if (act) st<VEC>(gx + row * ldgx + f, acc);
    }
}

// ---------------------------------------------------------------- dispatch
int pick_vec(int64_t F, std::initializer_list<std::pair<const void *, int64_t>> bufs) {
    for (int v : {4, 2}) {
        bool ok = (F % v) == 0;
        for (auto &b : bufs)
            ok = ok && (b.first == nullptr || (aligned(b.first, 4 * v) && (b.second % v) == 0));
        if (ok) return v;
    }
    return 1;
}

int pick_lpr(int64_t F, int vec) {
    const int64_t chunks = ceil_div(F, vec);
    int l = 4;
    while (l < 64 && l < chunks) l <<= 1;
    return l;
}

#define NGNN_LPR_SWITCH(LPRV, ...)                \
    switch (LPRV) {                               \
        case 4: {                                 \
            constexpr int LPR = 4;                \
            __VA_ARGS__;                          \
        } break;                                  \
        case 8: {                                 \
            constexpr int LPR = 8;                \
            __VA_ARGS__;                          \
        } break;                                  \
        case 16: {                                \
            constexpr int LPR = 16;               \
            __VA_ARGS__;                          \
        } break;                                  \
        case 32: {                                \
            constexpr int LPR = 32;               \
            __VA_ARGS__;                          \
        } break;                                  \
        default: {                                \
            constexpr int LPR = 64;               \
            __VA_ARGS__;                          \
        } break;                                  \
    }

#define NGNN_VEC_SWITCH(VECV, ...)   \
    switch (VECV) {                  \
        case 4: {                    \
            constexpr int VEC = 4;   \
            __VA_ARGS__;             \
        } break;                     \
        case 2: {                    \
            constexpr int VEC = 2;   \
            __VA_ARGS__;             \
        } break;                     \
        default: {                   \
            constexpr int VEC = 1;   \
            __VA_ARGS__;             \
        } break;                     \
    }

#define NGNN_RED_SWITCH(REDV, ...)                       \
    switch (REDV) {                                      \
        case NGNN_REDUCE_SUM: {                          \
            constexpr int RED = NGNN_REDUCE_SUM;         \
            __VA_ARGS__;                                 \
        } break;                                         \
        case NGNN_REDUCE_MEAN: {                         \
            constexpr int RED = NGNN_REDUCE_MEAN;        \
            __VA_ARGS__;                                 \
        } break;                                         \
        default: {                                       \
            constexpr int RED = NGNN_REDUCE_MAX;         \
            __VA_ARGS__;                                 \
        } break;                                         \
    }

}  // namespace
}  // namespace ngnn

using namespace ngnn;

extern "C" int ngnn_seg_agg_fwd(const void *x, int64_t ldx, int64_t F, const int32_t *rowptr,
                                const int32_t *col, int64_t n_dst, int reduce, int dtype, void *out,
                                int64_t ldo, void *stream) {
    NGNN_RETURN_IF(dtype != NGNN_F32 && dtype != NGNN_BF16, NGNN_E_DTYPE);
    NGNN_RETURN_IF(reduce < NGNN_REDUCE_SUM || reduce > NGNN_REDUCE_MAX, NGNN_E_ARG);
    NGNN_RETURN_IF(F < 0 || n_dst < 0 || !rowptr, NGNN_E_ARG);
    NGNN_RETURN_IF(ldx < F || ldo < F, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(F) || !fits_i32(n_dst), NGNN_E_RANGE);
    if (F == 0 || n_dst == 0) return NGNN_OK;
    // col may be NULL when the block has no edges (rowptr is all zeros then)
    NGNN_RETURN_IF(!x || !out, NGNN_E_ARG);
    if (dtype == NGNN_BF16) {  // bf16 rows: F and ldx multiples of 4, 8-B aligned
        NGNN_RETURN_IF(F % 4 != 0 || ldx % 4 != 0 || !aligned(x, 8), NGNN_E_SHAPE);
        const unsigned g = static_cast<unsigned>(ceil_div(n_dst, 4));
        const uint16_t *xb = static_cast<const uint16_t *>(x);
        float *of = static_cast<float *>(out);
        if (reduce == NGNN_REDUCE_MEAN)
            hipLaunchKernelGGL(k_seg_agg_fwd_bf16<NGNN_REDUCE_MEAN>, dim3(g), dim3(256), 0,
                               as_stream(stream), xb, ldx, (int)F, rowptr, col, (int)n_dst, of, ldo);
        else if (reduce == NGNN_REDUCE_SUM)
            hipLaunchKernelGGL(k_seg_agg_fwd_bf16<NGNN_REDUCE_SUM>, dim3(g), dim3(256), 0,
                               as_stream(stream), xb, ldx, (int)F, rowptr, col, (int)n_dst, of, ldo);
        else
            hipLaunchKernelGGL(k_seg_agg_fwd_bf16<NGNN_REDUCE_MAX>, dim3(g), dim3(256), 0,
                               as_stream(stream), xb, ldx, (int)F, rowptr, col, (int)n_dst, of, ldo);
        return launch_status();
    }
    const int vec = pick_vec(F, {{x, ldx}, {out, ldo}});
    const int lpr = pick_lpr(F, vec);
    const unsigned grid = static_cast<unsigned>(ceil_div(n_dst, 256 / lpr));
    hipStream_t st = as_stream(stream);
    const float *xf = static_cast<const float *>(x);
    float *of = static_cast<float *>(out);
    NGNN_RED_SWITCH(reduce, NGNN_VEC_SWITCH(vec, NGNN_LPR_SWITCH(lpr, {
        hipLaunchKernelGGL((k_seg_agg_fwd<VEC, LPR, RED>), dim3(grid), dim3(256), 0, st, xf, ldx,
                           (int)F, rowptr, col, (int)n_dst, of, ldo);
    })));
    return launch_status();
}

extern "C" size_t ngnn_seg_agg_bwd_workspace_bytes(int64_t n_dst, int64_t F, int reduce) {
    if (reduce != NGNN_REDUCE_MAX || n_dst <= 0 || F <= 0) return 0;
    return sizeof(float) * (size_t)n_dst * (size_t)F;
}

extern "C" int ngnn_seg_agg_bwd(const void *grad_out, int64_t ldg, int64_t F, const int32_t *rowptr,
                                const int32_t *col, int64_t n_dst, const int32_t *rowptr_t,
                                const int32_t *col_t, int64_t n_src, int reduce, int dtype,
                                const void *x, int64_t ldx, const void *agg, int64_t lda,
                                void *grad_x, int64_t ldgx, void *ws, size_t ws_bytes,
                                void *stream) {
    NGNN_RETURN_IF(dtype != NGNN_F32, NGNN_E_DTYPE);
    NGNN_RETURN_IF(reduce < NGNN_REDUCE_SUM || reduce > NGNN_REDUCE_MAX, NGNN_E_ARG);
    NGNN_RETURN_IF(F < 0 || n_dst < 0 || n_src < 0, NGNN_E_ARG);
    NGNN_RETURN_IF(ldg < F || ldgx < F, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(F) || !fits_i32(n_dst) || !fits_i32(n_src), NGNN_E_RANGE);
    if (F == 0 || n_src == 0) return NGNN_OK;
    NGNN_RETURN_IF(!grad_x || !rowptr_t || !rowptr, NGNN_E_ARG);  // col_t NULL iff no edges
    hipStream_t st = as_stream(stream);
    const float *gf = static_cast<const float *>(grad_out);
    float *gxf = static_cast<float *>(grad_x);
    if (reduce != NGNN_REDUCE_MAX) {
        const int vec = pick_vec(F, {{grad_out, ldg}, {grad_x, ldgx}});
        const int lpr = pick_lpr(F, vec);
        const unsigned grid = static_cast<unsigned>(ceil_div(n_src, 256 / lpr));
        NGNN_RED_SWITCH(reduce == NGNN_REDUCE_MEAN ? NGNN_REDUCE_MEAN : NGNN_REDUCE_SUM,
                        NGNN_VEC_SWITCH(vec, NGNN_LPR_SWITCH(lpr, {
                            if constexpr (RED != NGNN_REDUCE_MAX) {
                                hipLaunchKernelGGL((k_seg_agg_bwd_sum<VEC, LPR, RED>), dim3(grid),
                                                   dim3(256), 0, st, gf, ldg, (int)F, rowptr,
                                                   rowptr_t, col_t, (int)n_src, gxf, ldgx);
                            }
                        })));
        return launch_status();
    }
    NGNN_RETURN_IF(!x || !agg, NGNN_E_ARG);
    NGNN_RETURN_IF(ldx < F || lda < F, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!ws || ws_bytes < ngnn_seg_agg_bwd_workspace_bytes(n_dst, F, reduce),
                   NGNN_E_WORKSPACE);
    const float *xf = static_cast<const float *>(x);
    const float *af = static_cast<const float *>(agg);
    float *gdist = static_cast<float *>(ws);
    const int vec = pick_vec(F, {{grad_out, ldg}, {grad_x, ldgx}, {x, ldx}, {agg, lda}, {ws, F}});
    const int lpr = pick_lpr(F, vec);
    NGNN_VEC_SWITCH(vec, NGNN_LPR_SWITCH(lpr, {
        if (n_dst > 0)
            hipLaunchKernelGGL((k_max_bwd_dist<VEC, LPR>), dim3(ceil_div(n_dst, 256 / LPR)),
                               dim3(256), 0, st, gf, ldg, (int)F, rowptr, col, (int)n_dst, xf, ldx,
                               af, lda, gdist);
        hipLaunchKernelGGL((k_max_bwd_gather<VEC, LPR>), dim3(ceil_div(n_src, 256 / LPR)),
                           dim3(256), 0, st, gdist, (int)F, rowptr_t, col_t, (int)n_src, xf, ldx,
                           af, lda, gxf, ldgx);
    }));
    return launch_status();
}
