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
//   root phase, per 128-column chunk of K:
//     X chunk [64 x 128] fp32 HBM -> LDS, every load issued before the first
//     LDS write (8 x 16 B per lane in flight);  MFMA against packed W_r.
//   neighbour phase (only if the tile has in-edges), per chunk:
//     AGG chunk gathered into the SAME LDS buffer: one 32-lane group per row
//     walks its neighbour list in edge order (identical fp32 sequence to
//     ngnn_seg_agg_fwd => bit-identical aggregate); MFMA against packed W_l.
//     Tiles without in-edges (the last hop of a NeighborLoader block, ~90% of
//     its rows) skip the gather AND the W_l half of the GEMM.
//   epilogue: accumulators -> LDS in 128-column passes -> full-row 16-B
//     coalesced stores with bias, ReLU and hash-RNG dropout applied.
// LDS = one 64 x 132 fp32 buffer (33 KB) => 4 workgroups per CU.
// MFMA: v_mfma_f32_16x16x4_f32 (exact fp32, k-ordered fma chain); A from LDS
// (ds_read_b128, 4 k-steps per read), B from a fragment-ordered copy of the
// weights (ngnn_pack_weight, ~100 KB, L2-resident), prefetched one k-group
// ahead.
//
// Roofline: fp32 MFMA peak 157.3 TF; flops = 2*N*K*F_out (root) +
// 2*N_edge_rows*K*F_out (neighbour); HBM bytes = x (N*K*4) + gathered rows
// (E*K*4) + col/rowptr + out (N*F_out*4).
#include <cstdlib>

#include "ngnn_device.h"

namespace ngnn {
namespace {

constexpr int BM = kBM, KC = kKC, LDA = kLDA;
constexpr int LPR = 32;  // lanes per row in the gather

// Optional modes (all off when the pointers are NULL):
//   n_rows_dev : effective row count = min(n_rows, *n_rows_dev), read on the
//                device (backward passes whose row bound is never on the host)
//   agg_out    : tiles with in-edges also store their aggregate rows (saved
//                for the backward's weight gradient; tiles without edges store
//                nothing -- their rows have degree 0 and agg 0)
//   xmask      : stage x * (xmask > 0 ? xscale : 0) instead of x (the
//                ReLU/dropout backward fused into a dgrad GEMM's input)
struct Extra {
    const int32_t *n_rows_dev;
    float *agg_out;
    int64_t ld_agg;
    const float *xmask;
    int64_t ldm;
    float xscale;
    const uint64_t *seed_dev;  // XORed into the dropout seed (HIP-graph replays)
};

// ---- X rows [row0, row0+64) x [k0, k0+128) -> LDS, zero padded
__device__ __forceinline__ float masked(float v, float m, float scale) {
    return m > 0.0f ? v * scale : 0.0f;
}

template <bool VEC>
__device__ __forceinline__ void stage_x(float *s, const float *__restrict__ x, int64_t ldx,
                                        int64_t row0, int rows, int k0, int K,
                                        const float *__restrict__ xm, int64_t ldm, float xs) {
    if (VEC) {
        constexpr int PER = BM * (KC / 4) / 256;  // 8 float4 per thread
        float4 v[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int idx = threadIdx.x + u * 256;
            const int r = idx >> 5, c = (idx & 31) << 2;
            const int k = k0 + c;
            v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (r < rows && k < K) v[u] = *reinterpret_cast<const float4 *>(x + (row0 + r) * ldx + k);
        }
        if (xm) {
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int idx = threadIdx.x + u * 256;
                const int r = idx >> 5, c = (idx & 31) << 2;
                const int k = k0 + c;
                if (r < rows && k < K) {
                    const float4 m = *reinterpret_cast<const float4 *>(xm + (row0 + r) * ldm + k);
                    v[u].x = masked(v[u].x, m.x, xs);
                    v[u].y = masked(v[u].y, m.y, xs);
                    v[u].z = masked(v[u].z, m.z, xs);
                    v[u].w = masked(v[u].w, m.w, xs);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int idx = threadIdx.x + u * 256;
            *reinterpret_cast<float4 *>(s + (idx >> 5) * LDA + ((idx & 31) << 2)) = v[u];
        }
    } else {
        constexpr int PER = BM * KC / 256;  // 32 floats per thread
        float v[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int idx = threadIdx.x + u * 256;
            const int r = idx >> 7, c = idx & 127;
            const int k = k0 + c;
            v[u] = (r < rows && k < K) ? x[(row0 + r) * ldx + k] : 0.0f;
            if (xm && r < rows && k < K) v[u] = masked(v[u], xm[(row0 + r) * ldm + k], xs);
        }
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int idx = threadIdx.x + u * 256;
            s[(idx >> 7) * LDA + (idx & 127)] = v[u];
        }
    }
}

// ---- gather-reduce AGG rows [row0, row0+64) x [k0, k0+128) into LDS
// 8 groups of 32 lanes, one row per group at a time; lane owns 4 columns
// (VEC: 4 consecutive; else 4 strided by 32).  Edge order is kept per column.
template <bool VEC, int RED>
__device__ __forceinline__ void stage_agg(float *s, const float *__restrict__ x, int64_t ldx,
                                          const int32_t *__restrict__ rowptr,
                                          const int32_t *__restrict__ col, int64_t row0, int rows,
                                          int k0, int K) {
    const int lane = threadIdx.x & (LPR - 1);
    const int grp = threadIdx.x / LPR;
    constexpr int UNR = 8;
    const int c0 = VEC ? lane * 4 : lane;
    for (int r = grp; r < BM; r += 256 / LPR) {
        float acc[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = (RED == NGNN_REDUCE_MAX) ? -INFINITY : 0.0f;
        int beg = 0, end = 0;
        if (r < rows) {
            beg = rowptr[row0 + r];
            end = rowptr[row0 + r + 1];
        }
        for (int eb = beg; eb < end; eb += LPR) {
            const int n = min(LPR, end - eb);
            const int myc = lane < n ? col[eb + lane] : 0;
            for (int k = 0; k < n; k += UNR) {
                float v[UNR][4];
#pragma unroll
                for (int u = 0; u < UNR; ++u) {
                    const int cc = __shfl(myc, k + u, LPR);
                    const bool ok = k + u < n;
                    const float *src = x + static_cast<int64_t>(cc) * ldx + k0;
                    if (VEC) {
                        float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
                        if (ok && k0 + c0 < K) t = *reinterpret_cast<const float4 *>(src + c0);
                        v[u][0] = t.x; v[u][1] = t.y; v[u][2] = t.z; v[u][3] = t.w;
                    } else {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int c = c0 + 32 * i;
                            v[u][i] = (ok && k0 + c < K) ? src[c] : 0.0f;
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < UNR; ++u) {
                    if (k + u < n) {
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            acc[i] = (RED == NGNN_REDUCE_MAX) ? nanmax(acc[i], v[u][i])
                                                              : acc[i] + v[u][i];
                    }
                }
            }
        }
        const int deg = end - beg;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float a = acc[i];
            if (RED == NGNN_REDUCE_MEAN) a = a / static_cast<float>(deg > 1 ? deg : 1);
            if (RED == NGNN_REDUCE_MAX && deg == 0) a = 0.0f;
            const int c = VEC ? c0 + i : c0 + 32 * i;
            if (c < KC) s[r * LDA + c] = (k0 + c < K) ? a : 0.0f;  // padding stays exactly 0
        }
    }
}

// ---- acc += S[64 x kcp] . Wpack[kg0 .. kg0 + kcp/16)
template <int MTW, int NTW>
__device__ __forceinline__ void mfma_chunk(v4f (&acc)[MTW][NTW], const float *s,
                                           const v4f *__restrict__ wpack, int KG, int kg0, int nkg,
                                           int mbase, int nbase, int NT) {
    const int lane = threadIdx.x & 63;
    const int arow = lane & 15, acol = 4 * (lane >> 4);
    // B loads are unconditional (tiles past NT read the last valid tile; their
    // accumulators are never stored) so the compiler can count them and keep
    // the next k-group's fragments in flight behind a partial vmcnt.
    const v4f *wt[NTW];
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt)
        wt[nt] = wpack + (static_cast<int64_t>(min(nbase + nt, NT - 1)) * KG + kg0) * 64 + lane;
    // ping-pong register sets: the loads for k-group g+1 are issued (and pinned
    // with a scheduling barrier) before the MFMAs of group g, no register copies
    v4f b0[NTW], b1[NTW];
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) b0[nt] = wt[nt][0];
    auto step = [&](int kg, v4f(&cur)[NTW], v4f(&nxt)[NTW]) {
        const int kn = min(kg + 1, nkg - 1);  // last group re-reads: harmless, branch-free
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) nxt[nt] = wt[nt][kn * 64];
        v4f a[MTW];
#pragma unroll
        for (int mt = 0; mt < MTW; ++mt)
            a[mt] = *reinterpret_cast<const v4f *>(s + (mbase + mt * 16 + arow) * LDA + kg * 16 + acol);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
                for (int nt = 0; nt < NTW; ++nt)
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt][i], cur[nt][i],
                                                                       acc[mt][nt], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    };
    int kg = 0;
    for (; kg + 2 <= nkg; kg += 2) {
        step(kg, b0, b1);
        step(kg + 1, b1, b0);
    }
    if (kg < nkg) step(kg, b0, b1);
}

template <int MTW, int NTW, int RED, bool VEC>
__global__ __launch_bounds__(256, (MTW * NTW >= 32) ? 2 : ((MTW * NTW >= 16) ? 3 : 4)) void k_sage_fwd(
    const float *__restrict__ x, int64_t ldx, int K, int n_rows, const int32_t *__restrict__ rowptr,
    const int32_t *__restrict__ col, const v4f *__restrict__ wl, const v4f *__restrict__ wr, int KG,
    int Fo, float *__restrict__ out, int64_t ldo, Epi epi, int vec_out, Extra ex) {
    __shared__ __attribute__((aligned(16))) float s[BM * LDA];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr int WMW = 4 / MTW;  // waves along M
    const int wm = wave % WMW, wn = wave / WMW;
    const int mbase = wm * MTW * 16, nbase = wn * NTW;
    const int NT = (Fo + 15) >> 4;
    if (ex.n_rows_dev) n_rows = min(n_rows, *ex.n_rows_dev);
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * BM;
    if (row0 >= n_rows) return;  // uniform: whole workgroup leaves
    const int rows = static_cast<int>(min<int64_t>(BM, n_rows - row0));
    const bool has_edges = (wl != nullptr) && (rowptr[row0 + rows] > rowptr[row0]);

    v4f acc[MTW][NTW];
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) acc[mt][nt] = v4f{0.f, 0.f, 0.f, 0.f};

    bool first = true;
    for (int k0 = 0; k0 < K; k0 += KC) {
        const int nkg = (min(KC, K - k0) + 15) >> 4;
        if (!first) __syncthreads();
        first = false;
        stage_x<VEC>(s, x, ldx, row0, rows, k0, K, ex.xmask, ex.ldm, ex.xscale);
        __syncthreads();
        mfma_chunk<MTW, NTW>(acc, s, wr, KG, k0 >> 4, nkg, mbase, nbase, NT);
    }
    if (has_edges) {
        for (int k0 = 0; k0 < K; k0 += KC) {
            const int nkg = (min(KC, K - k0) + 15) >> 4;
            __syncthreads();
            stage_agg<VEC, RED>(s, x, ldx, rowptr, col, row0, rows, k0, K);
            __syncthreads();
            if (ex.agg_out) {  // save the aggregate for the backward (edge tiles only)
                const int kc = min(KC, K - k0);
                for (int idx = threadIdx.x; idx < rows * kc; idx += 256) {
                    const int r = idx / kc, c = idx - r * kc;
                    ex.agg_out[(row0 + r) * ex.ld_agg + k0 + c] = s[r * LDA + c];
                }
            }
            mfma_chunk<MTW, NTW>(acc, s, wl, KG, k0 >> 4, nkg, mbase, nbase, NT);
        }
    }

    // ---- epilogue straight from the accumulators (no LDS round trip, no
    // barrier): in a 16x16 C tile lane l holds rows 4*(l>>4)+j of column l&15,
    // so one store instruction writes four 64-B row segments; the neighbouring
    // n-tile completes each 128-B line in L2.
    const int q = lane >> 4, cl = lane & 15;
    (void)vec_out;
    if (ex.seed_dev) epi.drop.reseed(*ex.seed_dev);
    uint32_t rk[MTW][4];
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            rk[mt][j] = epi.drop.row_key(static_cast<uint32_t>(row0 + mbase + mt * 16 + 4 * q + j));
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
        const int c = (nbase + nt) * 16 + cl;
        if (c >= Fo) continue;
        const float bc = epi.bias ? epi.bias[c] : 0.0f;
#pragma unroll
        for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int r = mbase + mt * 16 + 4 * q + j;
                if (r >= rows) continue;
                float v = acc[mt][nt][j];
                if (epi.bias) v += bc;
                if (epi.relu) v = (v < 0.0f) ? 0.0f : v;  // NaN passes, like torch.relu
                if (epi.drop.thresh)
                    v = epi.drop.keep(rk[mt][j], epi.col_base + c) ? v * epi.drop.scale : 0.0f;
                out[(row0 + r) * ldo + c] = v;
            }
    }
}

// ---- weight packing: W [Fo, K] (PyG Linear layout, row-major, ld ldw) ->
// fragment-ordered float4 [NT][KG][64]: lane l, element i holds
// W[nt*16 + (l&15)][kg*16 + 4*(l>>4) + i]  (zero outside Fo x K)
// Generalised: the logical matrix M[Fo][K] is the row-concatenation of w0
// (rows [0, rows0)) and w1 (rows [rows0, Fo)); `trans` reads each source
// transposed (M[n][k] = src[k][n]) -- the dgrad GEMM of the backward uses
// M = [W_l^T ; W_r^T].
__global__ __launch_bounds__(256) void k_pack_weight(const float *__restrict__ w0,
                                                     const float *__restrict__ w1, int64_t ldw,
                                                     int rows0, int Fo, int K, int trans, int KG,
                                                     int NT, float *__restrict__ packed) {
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
    float v = 0.0f;
    if (n < Fo && k < K) {
        const float *src = n < rows0 ? w0 : w1;
        const int64_t nn = n < rows0 ? n : n - rows0;
        v = trans ? src[static_cast<int64_t>(k) * ldw + nn] : src[nn * ldw + k];
    }
    packed[idx] = v;
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

// ---- *r_next = max(*r_next, R, 1 + max col[0..rowptr[R])), R = *r_ptr;
// *nnz_out = rowptr[R] (nullable).  Rows of the input gradient that can be
// nonzero when the output gradient is zero past row R.
__global__ __launch_bounds__(256) void k_prefix_stats(const int32_t *__restrict__ rowptr,
                                                      const int32_t *__restrict__ col,
                                                      const int32_t *__restrict__ r_ptr,
                                                      int32_t *__restrict__ nnz_out,
                                                      int32_t *__restrict__ r_next) {
    const int R = *r_ptr;
    const int nnz = rowptr[R];
    int m = R;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nnz;
         e += (int64_t)gridDim.x * blockDim.x)
        m = max(m, col[e] + 1);
    for (int off = 32; off > 0; off >>= 1) m = max(m, __shfl_xor(m, off));
    __shared__ int sm;
    if (threadIdx.x == 0) sm = 0;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) atomicMax(&sm, m);
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicMax(r_next, sm);
        if (blockIdx.x == 0 && nnz_out) *nnz_out = nnz;
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

extern "C" int ngnn_pack_weight_ex(const float *w0, const float *w1, int64_t ldw, int64_t rows0,
                                   int64_t Fo, int64_t K, int transposed, void *packed,
                                   void *stream) {
    NGNN_RETURN_IF(Fo <= 0 || K <= 0 || !w0 || !packed || rows0 < 0 || rows0 > Fo, NGNN_E_ARG);
    NGNN_RETURN_IF(rows0 < Fo && !w1, NGNN_E_ARG);
    NGNN_RETURN_IF(transposed ? ldw < std::max<int64_t>(rows0, Fo - rows0) : ldw < K, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(Fo) || !fits_i32(K), NGNN_E_RANGE);
    const int NT = static_cast<int>(ceil_div(Fo, 16)), KG = static_cast<int>(ceil_div(K, 16));
    const int64_t total = static_cast<int64_t>(NT) * KG * 256;
    hipLaunchKernelGGL(k_pack_weight, dim3(ceil_div(total, 256)), dim3(256), 0, as_stream(stream),
                       w0, w1 ? w1 : w0, ldw, (int)rows0, (int)Fo, (int)K, transposed, KG, NT,
                       static_cast<float *>(packed));
    return launch_status();
}

extern "C" int ngnn_pack_weight(const float *w, int64_t ldw, int64_t Fo, int64_t K, void *packed,
                                void *stream) {
    return ngnn_pack_weight_ex(w, nullptr, ldw, Fo, Fo, K, 0, packed, stream);
}

#define NGNN_SAGE_CASE(MTW_, NTW_)                                                             \
    do {                                                                                       \
        auto launch = [&](auto red_c, auto vec_c) {                                            \
            constexpr int RED_ = decltype(red_c)::value;                                       \
            constexpr bool VEC_ = decltype(vec_c)::value;                                      \
            hipLaunchKernelGGL((k_sage_fwd<MTW_, NTW_, RED_, VEC_>), dim3(grid), dim3(256),    \
                               0, st, xf, ldx, (int)K, (int)n_rows, rowptr, col, wl, wr, KG,  \
                               (int)Fo, of, ldo, epi, vec_out, ex);                            \
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
                             const int32_t *n_rows_dev, const int32_t *rowptr, const int32_t *col,
                             int reduce, const void *wl_packed, const void *wr_packed,
                             const float *bias, int64_t Fo, float *out, int64_t ldo, int relu,
                             float p_drop, uint64_t seed, const uint64_t *seed_dev,
                             float *agg_out, int64_t ld_agg, const float *xmask, int64_t ldm,
                             float xscale, void *stream) {
    NGNN_RETURN_IF(reduce < NGNN_REDUCE_SUM || reduce > NGNN_REDUCE_MAX, NGNN_E_ARG);
    NGNN_RETURN_IF(K <= 0 || Fo <= 0 || n_rows < 0 || !wr_packed, NGNN_E_ARG);
    NGNN_RETURN_IF(wl_packed && !rowptr, NGNN_E_ARG);
    NGNN_RETURN_IF(ldx < K || ldo < Fo, NGNN_E_SHAPE);
    NGNN_RETURN_IF(agg_out && ld_agg < K, NGNN_E_SHAPE);
    NGNN_RETURN_IF(xmask && ldm < K, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(K) || !fits_i32(n_rows) || !fits_i32(Fo), NGNN_E_RANGE);
    NGNN_RETURN_IF(p_drop < 0.0f || !(p_drop <= 1.0f), NGNN_E_ARG);
    if (n_rows == 0) return NGNN_OK;
    NGNN_RETURN_IF(!x || !out, NGNN_E_ARG);
    if (!xmask) {  // default path: the row-tile kernel (ngnn_sage_rt.hip)
        int rc = NGNN_OK;
        if (sage_fwd_rowtile(x, ldx, K, n_rows, n_rows_dev, rowptr, col, reduce, wl_packed,
                             wr_packed, bias, Fo, out, ldo, relu, p_drop, seed, seed_dev, agg_out,
                             ld_agg, as_stream(stream), &rc))
            return rc;
    }
    const int vec_in = (K % 4 == 0) && (ldx % 4 == 0) && aligned(x, 16) &&
                       (!xmask || ((ldm % 4 == 0) && aligned(xmask, 16)));
    const int KG = static_cast<int>(ceil_div(K, 16));
    const unsigned grid = static_cast<unsigned>(ceil_div(n_rows, BM));
    hipStream_t st = as_stream(stream);
    const float *xf = x;
    // outputs wider than 512 columns: one launch per 512-column slice (the
    // packed weights are n-tile major, so a slice is a contiguous sub-array).
    // (Narrower slices for small grids -- 4 x 128 columns for Amazon-Computers'
    // 128-tile layer 0 -- were measured: 1.2 ms vs 0.47 ms, the per-slice x
    // staging and max re-gather cost more than the occupancy gains.)
    for (int64_t c0 = 0; c0 < Fo; c0 += 512) {
        const int64_t Fo_c = std::min<int64_t>(512, Fo - c0);
        const int64_t toff = (c0 / 16) * KG * 64;  // float4 offset of the slice's first n-tile
        Extra ex{n_rows_dev, c0 == 0 ? agg_out : nullptr, ld_agg, xmask, ldm, xscale, seed_dev};
        float *of = out + c0;
        const int vec_out = (Fo_c % 4 == 0) && (ldo % 4 == 0) && aligned(of, 16);
        const int NT = static_cast<int>(ceil_div(Fo_c, 16));
        Epi epi{bias ? bias + c0 : nullptr, relu, make_dropout(p_drop, seed), static_cast<int>(c0)};
        const v4f *wl = wl_packed ? static_cast<const v4f *>(wl_packed) + toff : nullptr;
        const v4f *wr = static_cast<const v4f *>(wr_packed) + toff;
        const int64_t Fo_arg = Fo_c;
        {
            const int64_t Fo = Fo_arg;  // the launch macro passes (int)Fo
            if (NT == 1) NGNN_SAGE_CASE(1, 1);
            else if (NT == 2) NGNN_SAGE_CASE(1, 2);
            else if (NT == 3) NGNN_SAGE_CASE(1, 3);
            else if (NT == 4) NGNN_SAGE_CASE(1, 4);
            else if (NT <= 8) NGNN_SAGE_CASE(2, 4);
            else if (NT <= 16) NGNN_SAGE_CASE(4, 4);
            else NGNN_SAGE_CASE(4, 8);
        }
        const int rc = launch_status();
        if (rc) return rc;
    }
    return NGNN_OK;
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

extern "C" int ngnn_block_prefix_stats(const int32_t *rowptr, const int32_t *col,
                                       const int32_t *r_ptr, int32_t *nnz_out, int32_t *r_next,
                                       int64_t E, void *stream) {
    NGNN_RETURN_IF(!rowptr || !r_ptr || !r_next || E < 0, NGNN_E_ARG);
    NGNN_RETURN_IF(!fits_i32(E), NGNN_E_RANGE);
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>(ceil_div(E > 0 ? E : 1, 256), 256));
    hipLaunchKernelGGL(k_prefix_stats, dim3(grid), dim3(256), 0, as_stream(stream), rowptr, col, r_ptr,
                       nnz_out, r_next);
    return launch_status();
}
