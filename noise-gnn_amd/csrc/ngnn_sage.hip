// Fused SAGEConv layer forward for gfx950: gather-aggregate into LDS, then
// fp32 MFMA for  out = act( [x | agg] . [W_r ; W_l]^T + b ).
//
// Replaces, for one layer of the reference's SAGE.forward (sage.py:33-39):
//   PyG SAGEConv.forward [ext]  = propagate (index_select + scatter mean)
//                                 -> lin_l(agg) + lin_r(x)
//   followed by x.relu() and F.dropout(p, training)   (sage.py:36-39)
// in ONE kernel: no [E,F] message tensor, no agg tensor in HBM, no separate
// bias / relu / dropout passes over the [N, F_out] activations.
//
// Work decomposition (one 256-thread workgroup = 64 target rows x all F_out):
//   1. X chunk  [64 x KC] fp32  HBM -> LDS (16-B coalesced row loads)
//   2. if the tile has in-edges: AGG chunk [64 x KC] gathered into LDS, one
//      32-lane group per row walking its neighbour list in edge order (the
//      same fp32 sequence as ngnn_seg_agg_fwd => bit-identical aggregate).
//      Tiles with no in-edges (the last hop of a NeighborLoader block, ~90%
//      of its rows) skip the gather AND the W_l half of the GEMM: agg = 0.
//   3. v_mfma_f32_16x16x4_f32 (exact fp32, k-ordered fma chain) over the chunk
//      with A from LDS (ds_read_b128) and B = pre-packed weights streamed from
//      L2 (each lane reads a contiguous 16 B of a fragment-ordered copy made by
//      ngnn_pack_weight; ~100 KB per matrix, resident in every XCD's L2).
//   4. epilogue through LDS so every output row is written with full-row
//      coalesced stores; bias, ReLU and dropout (counter-based hash RNG keyed by
//      (seed, row, col): the mask is never stored, backward reads y > 0).
//
// Roofline: fp32 MFMA peak 157.3 TF; 2*N*K*F_out flops for the
// root term + 2*N_edge_rows*K*F_out for the neighbour term.  HBM traffic is
// x (N*K*4) + gathered rows (E*K*4) + out (N*F_out*4).
#include "ngnn_internal.h"

namespace ngnn {
namespace {

typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int BM = 64;         // target rows per workgroup
constexpr int KC = 128;        // K chunk staged in LDS (floats)
constexpr int LDA = KC + 4;    // padded LDS row stride (floats)
constexpr int LPR = 32;        // lanes per row in the gather
constexpr int SMEM_FLOATS = 2 * BM * LDA;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// uniform in [0,1) from (seed, row, col); identical formula in ngnn_dropout_mask
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t row, uint32_t col) {
    const uint64_t h = mix64(seed ^ mix64((row << 20) ^ col));
    return static_cast<float>(h >> 40) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ float nanmax(float acc, float v) {
    return (acc != acc) ? acc : ((v != v || v > acc) ? v : acc);
}

struct Epi {
    const float *bias;
    int relu;
    float p;
    float scale;
    uint64_t seed;
    __device__ __forceinline__ float operator()(float v, int64_t row, int c) const {
        if (bias) v += bias[c];
        if (relu) v = (v < 0.0f) ? 0.0f : v;  // NaN passes, like torch.relu
        if (p > 0.0f) {
            if (p >= 1.0f) return 0.0f;
            v = (uniform01(seed, static_cast<uint64_t>(row), static_cast<uint32_t>(c)) >= p)
                    ? v * scale
                    : 0.0f;
        }
        return v;
    }
};

// ---- stage X rows [row0, row0+64) x [k0, k0+kcp) into LDS (zero padded)
template <bool VEC>
__device__ __forceinline__ void stage_x(float *sx, const float *__restrict__ x, int64_t ldx,
                                        int64_t row0, int rows, int k0, int kcp, int K) {
    if (VEC) {
        const int c4n = kcp >> 2;
        for (int idx = threadIdx.x; idx < BM * c4n; idx += 256) {
            const int r = idx / c4n, c = (idx - r * c4n) << 2;
            const int k = k0 + c;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (r < rows && k < K) v = *reinterpret_cast<const float4 *>(x + (row0 + r) * ldx + k);
            *reinterpret_cast<float4 *>(sx + r * LDA + c) = v;
        }
    } else {
        for (int idx = threadIdx.x; idx < BM * kcp; idx += 256) {
            const int r = idx / kcp, c = idx - r * kcp;
            const int k = k0 + c;
            sx[r * LDA + c] = (r < rows && k < K) ? x[(row0 + r) * ldx + k] : 0.0f;
        }
    }
}

// ---- gather-reduce AGG rows into LDS: 8 rows at a time, 32 lanes per row
template <bool VEC, int RED>
__device__ __forceinline__ void stage_agg(float *sa, const float *__restrict__ x, int64_t ldx,
                                          const int32_t *__restrict__ rowptr,
                                          const int32_t *__restrict__ col, int64_t row0, int rows,
                                          int k0, int kcp, int K) {
    const int lane = threadIdx.x & (LPR - 1);
    const int grp = threadIdx.x / LPR;  // 0..7
    constexpr int UNR = 4;
    for (int r = grp; r < BM; r += 256 / LPR) {
        float acc[4];
        const float init = (RED == NGNN_REDUCE_MAX) ? -INFINITY : 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = init;
        int beg = 0, end = 0;
        if (r < rows) {
            beg = rowptr[row0 + r];
            end = rowptr[row0 + r + 1];
        }
        // column set of this lane: VEC -> 4 consecutive (c0..c0+3), else 4 strided by 32
        const int c0 = VEC ? lane * 4 : lane;
        for (int eb = beg; eb < end; eb += LPR) {
            const int n = min(LPR, end - eb);
            const int myc = lane < n ? col[eb + lane] : 0;
            int k = 0;
            for (; k + UNR <= n; k += UNR) {
                int cc[UNR];
                float v[UNR][4];
#pragma unroll
                for (int u = 0; u < UNR; ++u) cc[u] = __shfl(myc, k + u, LPR);
#pragma unroll
                for (int u = 0; u < UNR; ++u) {
                    const float *src = x + static_cast<int64_t>(cc[u]) * ldx + k0;
                    if (VEC) {
                        float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
                        if (k0 + c0 < K) t = *reinterpret_cast<const float4 *>(src + c0);
                        v[u][0] = t.x; v[u][1] = t.y; v[u][2] = t.z; v[u][3] = t.w;
                    } else {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int c = c0 + 32 * i;
                            v[u][i] = (c < kcp && k0 + c < K) ? src[c] : 0.0f;
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < UNR; ++u)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        acc[i] = (RED == NGNN_REDUCE_MAX) ? nanmax(acc[i], v[u][i]) : acc[i] + v[u][i];
            }
            for (; k < n; ++k) {
                const int c1 = __shfl(myc, k, LPR);
                const float *src = x + static_cast<int64_t>(c1) * ldx + k0;
                float v[4];
                if (VEC) {
                    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (k0 + c0 < K) t = *reinterpret_cast<const float4 *>(src + c0);
                    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
                } else {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int c = c0 + 32 * i;
                        v[i] = (c < kcp && k0 + c < K) ? src[c] : 0.0f;
                    }
                }
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    acc[i] = (RED == NGNN_REDUCE_MAX) ? nanmax(acc[i], v[i]) : acc[i] + v[i];
            }
        }
        const int deg = end - beg;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float a = acc[i];
            if (RED == NGNN_REDUCE_MEAN) a = a / static_cast<float>(deg > 1 ? deg : 1);
            if (RED == NGNN_REDUCE_MAX && deg == 0) a = 0.0f;
            if (!VEC && !(c0 + 32 * i < kcp)) continue;
            if (VEC && c0 >= kcp) continue;
            // padded columns (k >= K) were summed as zeros: keep them exactly 0
            const int c = VEC ? c0 + i : c0 + 32 * i;
            sa[r * LDA + c] = (k0 + c < K) ? a : 0.0f;
        }
    }
}

template <int MTW, int NTW>
__device__ __forceinline__ void mfma_chunk(v4f (&acc)[MTW][NTW], const float *s,
                                           const v4f *__restrict__ wpack, int KG, int kg0,
                                           int kcp, int mbase, int nbase, int NT) {
    const int lane = threadIdx.x & 63;
    const int arow = lane & 15, acol = 4 * (lane >> 4);
    for (int kg = 0; kg < (kcp >> 4); ++kg) {
        v4f a[MTW], b[NTW];
#pragma unroll
        for (int mt = 0; mt < MTW; ++mt)
            a[mt] = *reinterpret_cast<const v4f *>(s + (mbase + mt * 16 + arow) * LDA + kg * 16 + acol);
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
            const int ntile = nbase + nt;
            b[nt] = (ntile < NT) ? wpack[(static_cast<int64_t>(ntile) * KG + kg0 + kg) * 64 + lane]
                                 : v4f{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
                for (int nt = 0; nt < NTW; ++nt)
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt][i], b[nt][i],
                                                                       acc[mt][nt], 0, 0, 0);
    }
}

template <int MTW, int NTW, int RED, bool VEC>
__global__ __launch_bounds__(256, 2) void k_sage_fwd(
    const float *__restrict__ x, int64_t ldx, int K, int n_rows, const int32_t *__restrict__ rowptr,
    const int32_t *__restrict__ col, const v4f *__restrict__ wl, const v4f *__restrict__ wr, int KG,
    int Fo, float *__restrict__ out, int64_t ldo, Epi epi, int vec_out) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *sx = smem;
    float *sa = smem + BM * LDA;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr int WMW = 4 / MTW;  // waves along M
    const int wm = wave % WMW, wn = wave / WMW;
    const int mbase = wm * MTW * 16, nbase = wn * NTW;
    const int NT = (Fo + 15) >> 4;
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * BM;
    const int rows = static_cast<int>(min<int64_t>(BM, n_rows - row0));
    const bool has_edges = (wl != nullptr) && (rowptr[row0 + rows] > rowptr[row0]);

    v4f acc[MTW][NTW];
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) acc[mt][nt] = v4f{0.f, 0.f, 0.f, 0.f};

    for (int k0 = 0; k0 < K; k0 += KC) {
        const int kc = min(KC, K - k0);
        const int kcp = (kc + 15) & ~15;
        if (k0 > 0) __syncthreads();  // previous chunk's MFMAs done reading LDS
        stage_x<VEC>(sx, x, ldx, row0, rows, k0, kcp, K);
        if (has_edges) stage_agg<VEC, RED>(sa, x, ldx, rowptr, col, row0, rows, k0, kcp, K);
        __syncthreads();
        mfma_chunk<MTW, NTW>(acc, sx, wr, KG, k0 >> 4, kcp, mbase, nbase, NT);
        if (has_edges) mfma_chunk<MTW, NTW>(acc, sa, wl, KG, k0 >> 4, kcp, mbase, nbase, NT);
    }

    // ---- epilogue
    const int q = lane >> 4, cl = lane & 15;
    if (NT * 16 + 4 <= 2 * LDA) {
        const int LDC = NT * 16 + 4;
        __syncthreads();  // all waves done with sx/sa
#pragma unroll
        for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
            for (int nt = 0; nt < NTW; ++nt) {
                const int ntile = nbase + nt;
                if (ntile >= NT) continue;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    smem[(mbase + mt * 16 + 4 * q + j) * LDC + ntile * 16 + cl] = acc[mt][nt][j];
            }
        __syncthreads();
        if (vec_out) {
            const int c4n = Fo >> 2;
            for (int idx = threadIdx.x; idx < rows * c4n; idx += 256) {
                const int r = idx / c4n, c = (idx - r * c4n) << 2;
                const int64_t row = row0 + r;
                const float *s = smem + r * LDC + c;
                float4 v;
                v.x = epi(s[0], row, c);
                v.y = epi(s[1], row, c + 1);
                v.z = epi(s[2], row, c + 2);
                v.w = epi(s[3], row, c + 3);
                *reinterpret_cast<float4 *>(out + row * ldo + c) = v;
            }
        } else {
            for (int idx = threadIdx.x; idx < rows * Fo; idx += 256) {
                const int r = idx / Fo, c = idx - r * Fo;
                const int64_t row = row0 + r;
                out[row * ldo + c] = epi(smem[r * LDC + c], row, c);
            }
        }
    } else {
#pragma unroll
        for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
            for (int nt = 0; nt < NTW; ++nt) {
                const int c = (nbase + nt) * 16 + cl;
                if (c >= Fo) continue;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int r = mbase + mt * 16 + 4 * q + j;
                    if (r < rows) out[(row0 + r) * ldo + c] = epi(acc[mt][nt][j], row0 + r, c);
                }
            }
    }
}

// ---- weight packing: W [Fo, K] (PyG Linear layout, row-major, ld ldw) ->
// fragment-ordered float4 [NT][KG][64]: lane l, element i holds
// W[nt*16 + (l&15)][kg*16 + 4*(l>>4) + i]  (zero outside Fo x K)
__global__ __launch_bounds__(256) void k_pack_weight(const float *__restrict__ w, int64_t ldw,
                                                     int Fo, int K, int KG, int NT,
                                                     float *__restrict__ packed) {
    const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t total = static_cast<int64_t>(NT) * KG * 64 * 4;
    if (idx >= total) return;
    const int i = idx & 3;
    const int lane = (idx >> 2) & 63;
    const int64_t t = idx >> 8;
    const int kg = static_cast<int>(t % KG);
    const int nt = static_cast<int>(t / KG);
    const int n = nt * 16 + (lane & 15);
    const int k = kg * 16 + 4 * (lane >> 4) + i;
    packed[idx] = (n < Fo && k < K) ? w[n * ldw + k] : 0.0f;
}

// ---- rows with any nonzero (or NaN): out[0] = max(out[0], 1 + last such row)
// Flat float4 sweep when rows are contiguous (ld == F), row-wise otherwise.
__global__ __launch_bounds__(256) void k_row_extent(const float *__restrict__ g, int64_t ld,
                                                    int64_t n_rows, int F, int32_t *__restrict__ out) {
    int64_t best = 0;
    const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
    if (ld == F && (reinterpret_cast<uintptr_t>(g) & 15) == 0) {
        const int64_t total = n_rows * F, n4 = total >> 2;
        const float4 *g4 = reinterpret_cast<const float4 *>(g);
        for (int64_t i = tid; i < n4; i += nthr) {
            const float4 v = g4[i];
            const int64_t e = 4 * i;
            if (v.w != 0.0f) best = max(best, (e + 3) / F + 1);
            else if (v.z != 0.0f) best = max(best, (e + 2) / F + 1);
            else if (v.y != 0.0f) best = max(best, (e + 1) / F + 1);
            else if (v.x != 0.0f) best = max(best, e / F + 1);
        }
        for (int64_t e = 4 * n4 + tid; e < total; e += nthr)
            if (g[e] != 0.0f) best = max(best, e / F + 1);
    } else {
        for (int64_t r = tid; r < n_rows; r += nthr) {
            bool nz = false;
            for (int c = 0; c < F; ++c) nz |= (g[r * ld + c] != 0.0f);
            if (nz) best = r + 1;
        }
    }
    int b = static_cast<int>(best);
    for (int off = 32; off > 0; off >>= 1) b = max(b, __shfl_xor(b, off));
    __shared__ int sbest;
    if (threadIdx.x == 0) sbest = 0;
    __syncthreads();
    if ((threadIdx.x & 63) == 0 && b) atomicMax(&sbest, b);
    __syncthreads();
    if (threadIdx.x == 0 && sbest) atomicMax(out, sbest);
}

// ---- status[1] = nnz = rowptr[R]; status[2] = max(R, 1 + max col[0..nnz))
__global__ __launch_bounds__(256) void k_prefix_stats(const int32_t *__restrict__ rowptr,
                                                      const int32_t *__restrict__ col, int64_t R_arg,
                                                      int32_t *__restrict__ status) {
    const int R = R_arg >= 0 ? static_cast<int>(R_arg) : status[0];
    const int nnz = rowptr[R];
    int m = R;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nnz;
         e += (int64_t)gridDim.x * blockDim.x)
        m = max(m, col[e] + 1);
    // wave max, then block max, then one atomic
    for (int off = 32; off > 0; off >>= 1) m = max(m, __shfl_xor(m, off));
    __shared__ int sm;
    if (threadIdx.x == 0) sm = 0;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) atomicMax(&sm, m);
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicMax(status + 2, sm);
        if (blockIdx.x == 0) {
            status[1] = nnz;
            if (R_arg >= 0) status[0] = R;
        }
    }
}

}  // namespace
}  // namespace ngnn

using namespace ngnn;

extern "C" size_t ngnn_pack_weight_bytes(int64_t Fo, int64_t K) {
    if (Fo <= 0 || K <= 0) return 0;
    return sizeof(float) * 4 * 64 * static_cast<size_t>(ceil_div(Fo, 16)) *
           static_cast<size_t>(ceil_div(K, 16));
}

extern "C" int ngnn_pack_weight(const float *w, int64_t ldw, int64_t Fo, int64_t K, void *packed,
                                void *stream) {
    NGNN_RETURN_IF(Fo <= 0 || K <= 0 || !w || !packed, NGNN_E_ARG);
    NGNN_RETURN_IF(ldw < K, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(Fo) || !fits_i32(K), NGNN_E_RANGE);
    const int NT = static_cast<int>(ceil_div(Fo, 16)), KG = static_cast<int>(ceil_div(K, 16));
    const int64_t total = static_cast<int64_t>(NT) * KG * 256;
    hipLaunchKernelGGL(k_pack_weight, dim3(ceil_div(total, 256)), dim3(256), 0, as_stream(stream), w,
                       ldw, (int)Fo, (int)K, KG, NT, static_cast<float *>(packed));
    return launch_status();
}

#define NGNN_SAGE_CASE(MTW_, NTW_)                                                             \
    do {                                                                                       \
        auto launch = [&](auto red_c, auto vec_c) {                                            \
            constexpr int RED_ = decltype(red_c)::value;                                       \
            constexpr bool VEC_ = decltype(vec_c)::value;                                      \
            hipLaunchKernelGGL((k_sage_fwd<MTW_, NTW_, RED_, VEC_>), dim3(grid), dim3(256),    \
                               SMEM_FLOATS * sizeof(float), st, xf, ldx, (int)K, (int)n_rows, \
                               rowptr, col, wl, wr, KG, (int)Fo, of, ldo, epi, vec_out);       \
        };                                                                                     \
        using T = std::true_type;                                                              \
        using Fb = std::false_type;                                                            \
        using RMEAN = std::integral_constant<int, NGNN_REDUCE_MEAN>;                           \
        using RSUM = std::integral_constant<int, NGNN_REDUCE_SUM>;                             \
        using RMAX = std::integral_constant<int, NGNN_REDUCE_MAX>;                             \
        if (reduce == NGNN_REDUCE_MEAN) {                                                      \
            if (vec_in) launch(RMEAN{}, T{}); else launch(RMEAN{}, Fb{});                      \
        } else if (reduce == NGNN_REDUCE_SUM) {                                                \
            if (vec_in) launch(RSUM{}, T{}); else launch(RSUM{}, Fb{});                        \
        } else {                                                                               \
            if (vec_in) launch(RMAX{}, T{}); else launch(RMAX{}, Fb{});                        \
        }                                                                                      \
    } while (0)

extern "C" int ngnn_sage_fwd(const float *x, int64_t ldx, int64_t K, int64_t n_rows,
                             const int32_t *rowptr, const int32_t *col, int reduce,
                             const void *wl_packed, const void *wr_packed, const float *bias,
                             int64_t Fo, float *out, int64_t ldo, int relu, float p_drop,
                             uint64_t seed, void *stream) {
    NGNN_RETURN_IF(reduce < NGNN_REDUCE_SUM || reduce > NGNN_REDUCE_MAX, NGNN_E_ARG);
    NGNN_RETURN_IF(K <= 0 || Fo <= 0 || n_rows < 0 || !rowptr || !wr_packed, NGNN_E_ARG);
    NGNN_RETURN_IF(ldx < K || ldo < Fo, NGNN_E_SHAPE);
    NGNN_RETURN_IF(Fo > 512, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(K) || !fits_i32(n_rows) || !fits_i32(Fo), NGNN_E_RANGE);
    NGNN_RETURN_IF(p_drop < 0.0f || !(p_drop <= 1.0f), NGNN_E_ARG);
    if (n_rows == 0) return NGNN_OK;
    NGNN_RETURN_IF(!x || !out, NGNN_E_ARG);
    const int vec_in = (K % 4 == 0) && (ldx % 4 == 0) && aligned(x, 16);
    const int vec_out = (Fo % 4 == 0) && (ldo % 4 == 0) && aligned(out, 16);
    const int NT = static_cast<int>(ceil_div(Fo, 16));
    const int KG = static_cast<int>(ceil_div(K, 16));
    Epi epi{bias, relu, p_drop, p_drop < 1.0f ? 1.0f / (1.0f - p_drop) : 0.0f, seed};
    const v4f *wl = static_cast<const v4f *>(wl_packed);
    const v4f *wr = static_cast<const v4f *>(wr_packed);
    const float *xf = x;
    float *of = out;
    const unsigned grid = static_cast<unsigned>(ceil_div(n_rows, BM));
    hipStream_t st = as_stream(stream);
    if (NT == 1) NGNN_SAGE_CASE(1, 1);
    else if (NT == 2) NGNN_SAGE_CASE(1, 2);
    else if (NT == 3) NGNN_SAGE_CASE(1, 3);
    else if (NT == 4) NGNN_SAGE_CASE(1, 4);
    else if (NT <= 8) NGNN_SAGE_CASE(2, 4);
    else if (NT <= 16) NGNN_SAGE_CASE(4, 4);
    else NGNN_SAGE_CASE(4, 8);
    return launch_status();
}

extern "C" int ngnn_row_extent(const float *g, int64_t ld, int64_t n_rows, int64_t F,
                               int32_t *out, void *stream) {
    NGNN_RETURN_IF(n_rows < 0 || F < 0 || !out, NGNN_E_ARG);
    NGNN_RETURN_IF(ld < F, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(n_rows) || !fits_i32(F), NGNN_E_RANGE);
    if (n_rows == 0 || F == 0) return NGNN_OK;
    NGNN_RETURN_IF(!g, NGNN_E_ARG);
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>(ceil_div(n_rows * F, 1024), 1024));
    hipLaunchKernelGGL(k_row_extent, dim3(grid), dim3(256), 0, as_stream(stream), g, ld, n_rows,
                       (int)F, out);
    return launch_status();
}

extern "C" int ngnn_block_prefix_stats(const int32_t *rowptr, const int32_t *col, int64_t R,
                                       int64_t E, int32_t *status, void *stream) {
    NGNN_RETURN_IF(!rowptr || !status || E < 0, NGNN_E_ARG);
    NGNN_RETURN_IF(!fits_i32(E), NGNN_E_RANGE);
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>(ceil_div(E > 0 ? E : 1, 256), 256));
    hipLaunchKernelGGL(k_prefix_stats, dim3(grid), dim3(256), 0, as_stream(stream), rowptr, col, R,
                       status);
    return launch_status();
}
