// Backward of one fused SAGE layer on gfx950, bounded by device-side row
// counts (no host round trip).
//
// The reference trains with loss = CE(model(x, ei)[:batch_size], y)
// (pipeline.py:155-160), so only the seed rows of the output gradient are
// nonzero.  R = the row bound of dz (device int), R' = rows of the input
// gradient that can be nonzero (ngnn_block_prefix_stats).  Everything below
// touches rows < R (weight gradients, dgrad GEMM) or rows < R' (gather).
//
//   ngnn_sage_wgrad        dW_r = dz^T h, dW_l = dz^T agg, db = sum dz
//     k_wgrad_partial: 512-thread workgroups, grid (slice, K-chunk of 128,
//       Fo-chunk of 64) ~ one workgroup per CU; slice s owns rows [rb, re),
//       an even 4-row-granular share of R, walked in 64-row chunks.  Per chunk
//       dz [64 x 64], h and agg [64 x 128] are loaded into registers (the
//       next chunk's loads overlap this chunk's MFMAs), written row-major to
//       LDS, and v_mfma_f32_16x16x4_f32 reduces over the rows (A = dz^T read as
//       ds_read_b32 columns, B = h / agg rows); waves 0-3 own dW_r tiles,
//       waves 4-7 dW_l tiles.  Partials -> ws slabs.  Splitting Fo (not only
//       rows) keeps the slab count, hence the slab write + reduce traffic, at
//       a quarter of a rows-only split for the products hidden layer.
//     k_wgrad_reduce: fixed-order slab sum => bitwise reproducible.
//   ngnn_sage_dgrad_gather dh = [j<R] dz W_r + transposed aggregation of dz W_l
//     over the source-grouped CSR, in edge order, edges into rows >= R skipped.
#include "ngnn_device.h"

namespace ngnn {
namespace {

constexpr int WG_BM = 64;       // rows per chunk
constexpr int WG_KC = 128;      // K columns per workgroup (grid.y)
constexpr int WG_NC = 64;       // Fo columns per workgroup (grid.z)
constexpr int LDZ = WG_NC + 16; // LDS strides: +16 floats keeps the two 16-lane
constexpr int LDH = WG_KC + 16; // row groups of a b32 read on disjoint banks
constexpr int S_MAX = 256;      // slices (partial slabs)

__host__ __device__ inline size_t slab_floats(int64_t Fo, int64_t K) {
    return static_cast<size_t>(2 * Fo * K + Fo);
}

// slices used for R rows: at most the launched S, at least ~64 rows each
__device__ __forceinline__ int wgrad_slices(int R, int S) {
    return max(1, min(S, (R + WG_BM - 1) / WG_BM));
}

// One 64-row chunk of one operand, COLS columns wide, held in registers by
// the 512 threads of a workgroup (a fixed number of loads per thread), so the
// next chunk's loads are in flight while the MFMAs of this one run.  Loads go
// through a buffer resource over rows [c0, re): rows >= re and columns >= K
// read 0 with no branches (a column past K gets an out-of-range offset).  The
// optional per-element mask (y > 0: ReLU/dropout of the forward) and per-row
// "has in-edges" test (rowptr: the saved aggregate of an edgeless row is never
// written) are applied when the registers are written to LDS, so no load
// waits on another.  Needs ld * 64 * 4 < 2^31 (host-checked).
template <int COLS, bool VEC, int MASK, bool DEG, bool BF = false>
struct Chunk {  // BF: the operand is bf16 (widened exactly when loaded); MASK: 0
                // none, 1 fp32 mask rows, 2 bf16 mask rows (a bf16 model's activations)
    static constexpr int W = VEC ? 4 : 1;
    static constexpr int CPR = COLS / W;               // loads per row
    static constexpr int N = WG_BM * CPR / 512;        // loads per thread
    static_assert(N >= 1 && (WG_BM * CPR) % 512 == 0, "chunk must tile the workgroup");
    using T = std::conditional_t<VEC, v4f, float>;
    T v[BF && VEC ? 1 : N];
    // bf16 quads stay packed until store(): widening them in load() would
    // make every load wait at once (the next chunk's loads must stay in
    // flight under this chunk's MFMAs)
    i32x2 raw[BF && VEC ? N : 1];
    T m[MASK == 1 ? N : 1];
    i32x2 mraw[MASK == 2 && VEC ? N : 1];  // bf16 mask quads, widened in store()
    float mh[MASK == 2 && !VEC ? N : 1];
    int d0[DEG ? N : 1], d1[DEG ? N : 1];

    // ridx (nullable): row r of the operand is row ridx[r] of src, a table of
    // src_rows rows (the fused x[n_id] gather of layer 0; < 2 GiB)
    __device__ __forceinline__ void load(const float *__restrict__ src, int64_t ld,
                                         const float *__restrict__ mask, int64_t ldm,
                                         const int32_t *__restrict__ rowptr, int64_t c0, int re,
                                         int k0, int K, const int64_t *__restrict__ ridx = nullptr,
                                         int64_t src_rows = 0) {
        constexpr uint32_t EB = BF ? 2u : 4u;
        const uint32_t nr = static_cast<uint32_t>(re - c0);
        const char *sb = reinterpret_cast<const char *>(src);
        const i32x4 rs = ridx ? make_rsrc(sb, static_cast<uint32_t>(src_rows * ld * EB))
                             : make_rsrc(sb + c0 * ld * EB, nr * static_cast<uint32_t>(ld) * EB);
        i32x4 rm = rs, rp = rs;
        constexpr uint32_t MB = MASK == 2 ? 2u : 4u;
        if (MASK) rm = make_rsrc(reinterpret_cast<const char *>(mask) + c0 * ldm * MB,
                                 nr * static_cast<uint32_t>(ldm) * MB);
        if (DEG) rp = make_rsrc(rowptr + c0, (nr + 1u) * 4u);
#pragma unroll
        for (int u = 0; u < N; ++u) {
            const int idx = static_cast<int>(threadIdx.x) + u * 512;
            const int r = idx / CPR, c = (idx % CPR) * W;
            const int k = k0 + c;
            const bool kok = k < K;
            int vo;
            if (ridx) {
                const int pr = r < static_cast<int>(nr) ? static_cast<int>(gload(ridx, c0 + r)) : -1;
                vo = (kok && pr >= 0) ? (pr * static_cast<int>(ld) + k) * static_cast<int>(EB) : kBufOOB;
            } else {
                vo = kok ? (r * static_cast<int>(ld) + k) * static_cast<int>(EB) : kBufOOB;
            }
            if constexpr (BF && VEC) {
                raw[u] = buf_load2i(rs, vo, 0, 0);
            } else if constexpr (BF) {  // the dword holding the element, then its half
                const int w = buf_load1i(rs, vo & ~3, 0, 0);
                v[u] = __int_as_float((vo & 2) ? (w & static_cast<int>(0xffff0000u)) : (w << 16));
            } else if constexpr (VEC) {
                if (!kok || k + 4 <= K) {
                    v[u] = buf_load4(rs, vo, 0, 0);
                } else {  // (K % 4 != 0: the row's last quad, element by element -- a
                          // 16-B load would straddle the next row / the range's end)
#pragma unroll
                    for (int i = 0; i < 4; ++i) v[u][i] = buf_load1(rs, k + i < K ? vo + 4 * i : kBufOOB, 0, 0);
                }
            } else {
                v[u] = buf_load1(rs, vo, 0, 0);
            }
            if (MASK) {
                const int mo = kok ? (r * static_cast<int>(ldm) + k) * static_cast<int>(MB) : kBufOOB;
                if constexpr (MASK == 2 && VEC) {
                    mraw[u] = buf_load2i(rm, mo, 0, 0);
                } else if constexpr (MASK == 2) {
                    const int w = buf_load1i(rm, mo & ~3, 0, 0);
                    mh[u] = __int_as_float((mo & 2) ? (w & static_cast<int>(0xffff0000u)) : (w << 16));
                } else if constexpr (VEC) {
                    m[u] = buf_load4(rm, mo, 0, 0);
                } else {
                    m[u] = buf_load1(rm, mo, 0, 0);
                }
            }
            if (DEG) {
                d0[u] = buf_load1i(rp, r * 4, 0, 0);
                d1[u] = buf_load1i(rp, r * 4 + 4, 0, 0);
            }
        }
    }

    __device__ __forceinline__ void store(float *lds, int ldl, float mscale) const {
#pragma unroll
        for (int u = 0; u < N; ++u) {
            const int idx = static_cast<int>(threadIdx.x) + u * 512;
            const int r = idx / CPR, c = (idx % CPR) * W;
            T w;
            if constexpr (BF && VEC) w = bf16x4_to_f32(raw[u]);
            else w = v[u];
            float *wf = reinterpret_cast<float *>(&w);
            T mv;
            if constexpr (MASK == 2 && VEC) mv = bf16x4_to_f32(mraw[u]);
            else if constexpr (MASK == 2) mv = mh[u];
            else mv = m[MASK ? u : 0];
            const float *mf = reinterpret_cast<const float *>(&mv);
#pragma unroll
            for (int i = 0; i < W; ++i) {
                float x = wf[i];
                if (MASK) x = mf[i] > 0.f ? x * mscale : 0.f;
                if (DEG) x = d1[u] > d0[u] ? x : 0.f;
                wf[i] = x;
            }
            *reinterpret_cast<T *>(lds + r * ldl + c) = w;
        }
    }

    // X3 staging (VEC only): the masked values as three bf16 parts (round to
    // nearest: v - p1 - p2 - p3 <= 2^-24 |v|) into the images img[0..NP) of
    // row stride ld (bf16 elements); NP == 1 for bf16 rows (exact in one
    // part, stored as loaded)
    // kq0 = K - k0: columns of the chunk that are real -- a 16-B load at a
    // 4-B aligned row start (K % 4 != 0) reads past K into the next row, and
    // those elements are zeroed here
    template <int NP>
    __device__ __forceinline__ void store_parts(__bf16 *img0, __bf16 *img1, __bf16 *img2, int ld,
                                                float mscale, int kq0 = 1 << 30) const {
        static_assert(VEC, "16-B staging");
#pragma unroll
        for (int u = 0; u < N; ++u) {
            const int idx = static_cast<int>(threadIdx.x) + u * 512;
            const int r = idx / CPR, c = (idx % CPR) * W;
            if constexpr (NP == 1 && BF && !MASK && !DEG) {
                *reinterpret_cast<i32x2 *>(img0 + r * ld + c) = raw[u];
                continue;
            }
            T w;
            if constexpr (BF) w = bf16x4_to_f32(raw[u]);
            else w = v[u];
            T mv;
            if constexpr (MASK == 2) mv = bf16x4_to_f32(mraw[u]);
            else mv = m[MASK ? u : 0];
            typedef __bf16 b4 __attribute__((ext_vector_type(4)));
            b4 p1, p2, p3;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float x = w[i];
                if (MASK) x = mv[i] > 0.f ? x * mscale : 0.f;
                if (DEG) x = d1[u] > d0[u] ? x : 0.f;
                if (c + i >= kq0) x = 0.f;
                const __bf16 h1 = static_cast<__bf16>(x);
                const float r1 = x - static_cast<float>(h1);
                const __bf16 h2 = static_cast<__bf16>(r1);
                p1[i] = h1;
                p2[i] = h2;
                p3[i] = static_cast<__bf16>(r1 - static_cast<float>(h2));
            }
            *reinterpret_cast<b4 *>(img0 + r * ld + c) = p1;
            if constexpr (NP > 1) {
                *reinterpret_cast<b4 *>(img1 + r * ld + c) = p2;
                *reinterpret_cast<b4 *>(img2 + r * ld + c) = p3;
            }
        }
    }
};

// the MFMAs of one staged chunk: nks 4-row k-steps, KTN (<= KTW) live K tiles
template <int NTW, int KTW, int KTN>
__device__ __forceinline__ void wgrad_mfma(v4f (&acc)[NTW][KTW], const float *sz, const float *sb,
                                           int nks, int nt0, int kt0, int i16, int kk) {
    // software-pipelined: the LDS reads of k-step ks+1 are issued before the
    // MFMAs of k-step ks (the last prefetch re-reads a valid row, unused)
    float a[NTW], b[KTN];
    auto fetch = [&](int ks, float(&fa)[NTW], float(&fb)[KTN]) {
        const int rr = ks * 4 + kk;
#pragma unroll
        for (int t = 0; t < NTW; ++t) fa[t] = sz[rr * LDZ + (nt0 + t) * 16 + i16];
#pragma unroll
        for (int t = 0; t < KTN; ++t) fb[t] = sb[rr * LDH + (kt0 + t) * 16 + i16];
    };
    fetch(0, a, b);
    for (int ks = 0; ks < nks; ++ks) {
        float an[NTW], bn[KTN];
        fetch(min(ks + 1, WG_BM / 4 - 1), an, bn);
#pragma unroll
        for (int ta = 0; ta < NTW; ++ta)
#pragma unroll
            for (int tb = 0; tb < KTN; ++tb)
                acc[ta][tb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[ta], b[tb], acc[ta][tb], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < NTW; ++t) a[t] = an[t];
#pragma unroll
        for (int t = 0; t < KTN; ++t) b[t] = bn[t];
    }
}

template <int NTW, int KTW, int KTN>
__device__ __forceinline__ void wgrad_mfma_dispatch(int ktn, v4f (&acc)[NTW][KTW], const float *sz,
                                                    const float *sb, int nks, int nt0, int kt0,
                                                    int i16, int kk) {
    if (ktn == KTN) wgrad_mfma<NTW, KTW, KTN>(acc, sz, sb, nks, nt0, kt0, i16, kk);
    else if constexpr (KTN > 1) wgrad_mfma_dispatch<NTW, KTW, KTN - 1>(ktn, acc, sz, sb, nks, nt0, kt0, i16, kk);
}

// NTW n-tiles x KTW k-tiles of 16x16 per wave.  SPLIT_N: the 4 waves of a
// matrix split the (4) Fo tiles of the workgroup; else they split the K tiles.
// Slice s owns rows [rb, re) (R split into S ranges on 4-row boundaries, so
// every used slice gets the same work +-4 rows), walked in 64-row chunks.
template <int NTW, int KTW, bool SPLIT_N, bool VZ, int VH, int MASK>
__global__ __launch_bounds__(512, 1) void k_wgrad_partial(
    const float *__restrict__ dy, int64_t ldy, const float *__restrict__ y, int64_t ldyy,
    float yscale, const float *__restrict__ h_arg, const float *const *h_dev, int64_t ldh,
    const int64_t *h_idx_arg, const int64_t *const *h_idx_dev, int64_t h_rows,
    const float *__restrict__ agg, int64_t ld_agg, const int32_t *__restrict__ rowptr,
    const int32_t *__restrict__ r_ptr, int Fo, int K, float *__restrict__ ws) {
    __shared__ __attribute__((aligned(16))) float smem[WG_BM * LDZ + 2 * WG_BM * LDH];  // 94 KB
    const float *__restrict__ h = h_dev ? *h_dev : h_arg;  // run-time address (graph slot)
    const int64_t *h_idx = h_idx_dev ? *h_idx_dev : h_idx_arg;  // fused x[n_id] (layer 0)
    float *sz = smem;                       // [64][LDZ]
    float *sh = sz + WG_BM * LDZ;           // [64][LDH]
    float *sa = sh + WG_BM * LDH;           // [64][LDH]
    const int R = *r_ptr;
    const int S = wgrad_slices(R, gridDim.x);
    const int s = blockIdx.x;
    if (s >= S) return;  // slab never read
    const int R4 = (R + 3) >> 2;
    const int rb = 4 * static_cast<int>(static_cast<int64_t>(s) * R4 / S);
    const int re = min(R, 4 * static_cast<int>(static_cast<int64_t>(s + 1) * R4 / S));
    const int k0 = blockIdx.y * WG_KC;
    const int n0 = blockIdx.z * WG_NC;
    const int kc = min(WG_KC, K - k0);
    const int nc = min(WG_NC, Fo - n0);
    const int KT = (kc + 15) >> 4;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int mat = wave >> 2;  // 0: dW_r (B = h), 1: dW_l (B = agg)
    const int w4 = wave & 3;
    const int nt0 = SPLIT_N ? w4 * NTW : 0;
    const int kt0 = SPLIT_N ? 0 : w4 * KTW;
    const int ktn = max(0, min(KTW, KT - kt0));  // live K tiles of this wave (uniform)
    const int i16 = lane & 15, kk = lane >> 4;
    const bool do_bias = blockIdx.y == 0;

    v4f acc[NTW][KTW];
#pragma unroll
    for (int a = 0; a < NTW; ++a)
#pragma unroll
        for (int b = 0; b < KTW; ++b) acc[a][b] = v4f{0.f, 0.f, 0.f, 0.f};
    // column sums of dz: thread (row group wave, column lane) over 8 rows/chunk
    float dbias = 0.0f;

    // VH: 0 scalar fp32, 1 16-B fp32, 2 bf16 h (8-B loads; agg stays fp32)
    Chunk<WG_NC, VZ, MASK, false> cz;
    Chunk<WG_KC, VH != 0, false, false, VH == 2> ch;
    Chunk<WG_KC, VH != 0, false, true> ca;
    if (rb < re) {
        cz.load(dy, ldy, y, ldyy, nullptr, rb, re, n0, Fo);
        ch.load(h, ldh, nullptr, 0, nullptr, rb, re, k0, K, h_idx, h_rows);
        ca.load(agg, ld_agg, nullptr, 0, rowptr, rb, re, k0, K);
    }
    for (int c0 = rb; c0 < re; c0 += WG_BM) {
        __syncthreads();  // the previous chunk's MFMAs are done with LDS
        cz.store(sz, LDZ, yscale);
        ch.store(sh, LDH, 1.0f);
        ca.store(sa, LDH, 1.0f);
        __syncthreads();
        const int c1 = c0 + WG_BM;
        if (c1 < re) {  // next chunk's loads overlap this chunk's MFMAs
            cz.load(dy, ldy, y, ldyy, nullptr, c1, re, n0, Fo);
            ch.load(h, ldh, nullptr, 0, nullptr, c1, re, k0, K, h_idx, h_rows);
            ca.load(agg, ld_agg, nullptr, 0, rowptr, c1, re, k0, K);
        }
        const int nks = min(WG_BM / 4, (re - c0 + 3) >> 2);
        if (do_bias) {
#pragma unroll
            for (int r = 0; r < 8; ++r) dbias += sz[(wave * 8 + r) * LDZ + lane];
        }
        const float *sb = mat ? sa : sh;
        // wave-uniform dispatch on the live K tiles (no per-MFMA branches)
        wgrad_mfma_dispatch<NTW, KTW, KTW>(ktn, acc, sz, sb, nks, nt0, kt0, i16, kk);
    }
    // ---- partial slab: [Pr Fo x K][Pl Fo x K][Pb Fo]; buffer stores, lanes
    // past Fo / K get an out-of-range offset (dropped)
    float *slab = ws + static_cast<size_t>(s) * slab_floats(Fo, K);
    const i32x4 prs = make_rsrc(slab + static_cast<size_t>(mat) * Fo * K,
                                static_cast<uint32_t>(Fo) * static_cast<uint32_t>(K) * 4u);
#pragma unroll
    for (int ta = 0; ta < NTW; ++ta)
#pragma unroll
        for (int tb = 0; tb < KTW; ++tb) {
            const int k = k0 + (kt0 + tb) * 16 + i16;
            const bool kok = k < K && kt0 + tb < KT;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int n = n0 + (nt0 + ta) * 16 + 4 * kk + j;
                const int off = (kok && n < n0 + nc) ? (n * K + k) * 4 : kBufOOB;
                buf_store1(acc[ta][tb][j], prs, off, 0, 0);
            }
        }
    if (do_bias) {
        __syncthreads();  // every wave is past its last LDS read
        smem[wave * 64 + lane] = dbias;
        __syncthreads();
        if (wave == 0 && lane < nc) {
            float t = 0.0f;
#pragma unroll
            for (int g = 0; g < 8; ++g) t += smem[g * 64 + lane];
            slab[2 * static_cast<size_t>(Fo) * K + n0 + lane] = t;
        }
    }
}

// ---- the weight gradient on bf16 MFMA (X3), Fo >= 64 with 16-B rows: the
// grid, slices and slab layout of k_wgrad_partial (k_wgrad_reduce unchanged).
// Per 64-row chunk the operands are staged in LDS as bf16 parts (dz and agg:
// three, RNE split3; h: three, or one for bf16 rows), and wave (mat = w >> 2,
// Fo tile w & 3) multiplies over the rows with v_mfma_f32_16x16x32_bf16 --
// A = dz^T, B = h (mat 0) / agg (mat 1), both through transposed LDS reads
// (ds_read_b64_tr_b16) in the row order {4q .. 4q+3, 16+4q .. 16+4q+3} of
// each 32-row step.  fp32 x fp32: the six products of the X3 forward
// (v1w1, v1w2, v2w1, v2w2, v1w3, v3w1; the dropped ones <= 2^-26 relative,
// each product exact in fp32), one-part bf16 h: three.  Against the exact
// 16x16x4 f32 steps: 16 vs 256 cycles per 32 rows and product.  db (column
// sums of dz) rides on the mat-0 waves as three more MFMAs per step against
// a ones operand.
constexpr int X3H = WG_KC + 16;  // LDS row strides (bf16): 72 dwords (and 40 / 72 for dz, below),
                                 // odd multiples of 8 -- transposed reads conflict-free
typedef __attribute__((address_space(3))) __bf16 LB16;
typedef short s4w __attribute__((ext_vector_type(4)));
typedef short s8w __attribute__((ext_vector_type(8)));
typedef __bf16 b8w __attribute__((ext_vector_type(8)));

// the MFMA operand of 32 rows x 16 columns c0 .. + 15 of a [rows][stride]
// bf16 image: lane (q, i) holds column c0 + i of rows 4q .. 4q+3, 16+4q ..
__device__ __forceinline__ b8w x3_frag(const LB16 *img, int stride, int c0, int ln) {
    const int q = ln >> 4, i = ln & 15;
    const LB16 *p = img + (4 * q + (i >> 2)) * stride + c0 + 4 * (i & 3);
    const s4w a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4w *)(p));
    const s4w b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4w *)(p + 16 * stride));
    const s8w v{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    return __builtin_bit_cast(b8w, v);
}

// NFW: Fo tiles per wave -- a workgroup covers 64 NFW columns of Fo, so the
// h / agg rows are read ceil(Fo / 64 NFW) times (NFW 2: half the re-reads of
// the products layers' 256-wide Fo; bf16 h only, where the images fit in LDS)
template <bool HB, int MASK, int NFW>
__global__ __launch_bounds__(512, 1) void k_wgrad_x3(
    const float *__restrict__ dy, int64_t ldy, const float *__restrict__ y, int64_t ldyy,
    float yscale, const float *__restrict__ h_arg, const float *const *h_dev, int64_t ldh,
    const int64_t *h_idx_arg, const int64_t *const *h_idx_dev, int64_t h_rows,
    const float *__restrict__ agg, int64_t ld_agg, const int32_t *__restrict__ rowptr,
    const int32_t *__restrict__ r_ptr, int Fo, int K, float *__restrict__ ws, int S_l, int GY, int GZ) {
    constexpr int NPH = HB ? 1 : 3;
    constexpr int WNC = WG_NC * NFW;  // Fo columns per workgroup
    constexpr int X3Z = WNC + 16;
    extern __shared__ __attribute__((aligned(16))) __bf16 x3s[];
    __bf16 *zi = x3s;                              // [3][64][X3Z]
    __bf16 *hi = zi + 3 * WG_BM * X3Z;             // [NPH][64][X3H]
    __bf16 *ai = hi + NPH * WG_BM * X3H;           // [3][64][X3H]
    const float *__restrict__ h = h_dev ? *h_dev : h_arg;
    const int64_t *h_idx = h_idx_dev ? *h_idx_dev : h_idx_arg;
    // 1-D grid, XCD-grouped (workgroup L runs on XCD L mod 8): the GZ Fo
    // chunks of one (row slice, K chunk) pair -- the workgroups that read the
    // same h / agg rows -- share an XCD and so its L2, instead of landing on
    // four of them (Amazon-Computers' S = 5, GY = 6: a pair's chunks were 30
    // ids apart); pair ids padded to a multiple of 8 (the padding exits)
    const int L = blockIdx.x, r8 = L >> 3;
    const int pr = (r8 / GZ) * 8 + (L & 7), zc = r8 % GZ;
    if (pr >= S_l * GY) return;
    const int R = *r_ptr;
    const int S = wgrad_slices(R, S_l);
    const int s = pr % S_l;
    if (s >= S) return;
    const int R4 = (R + 3) >> 2;
    const int rb = 4 * static_cast<int>(static_cast<int64_t>(s) * R4 / S);
    const int re = min(R, 4 * static_cast<int>(static_cast<int64_t>(s + 1) * R4 / S));
    const int k0 = (pr / S_l) * WG_KC;
    const int n0 = zc * WNC;
    const int kc = min(WG_KC, K - k0);
    const int nc = min(WNC, Fo - n0);
    const int KT = __builtin_amdgcn_readfirstlane((kc + 15) >> 4);
    const int wv = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int ln = threadIdx.x & 63;
    const int mat = wv >> 2, w4 = wv & 3;
    const bool do_bias = k0 == 0 && mat == 0;

    v4f acc[NFW][8], accb[NFW];
#pragma unroll
    for (int f = 0; f < NFW; ++f) {
        accb[f] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[f][b] = v4f{0.f, 0.f, 0.f, 0.f};
    }
    b8w ones;
#pragma unroll
    for (int j = 0; j < 8; ++j) ones[j] = static_cast<__bf16>(1.0f);

    Chunk<WNC, true, MASK, false> cz;
    Chunk<WG_KC, true, false, false, HB> ch;
    Chunk<WG_KC, true, false, true> ca;
    if (rb < re) {
        cz.load(dy, ldy, y, ldyy, nullptr, rb, re, n0, Fo);
        ch.load(h, ldh, nullptr, 0, nullptr, rb, re, k0, K, h_idx, h_rows);
        ca.load(agg, ld_agg, nullptr, 0, rowptr, rb, re, k0, K);
    }
    const LB16 *lz = (const LB16 *)(zi), *lh = (const LB16 *)(hi), *la = (const LB16 *)(ai);
    // the chunk loop, one copy per B-operand part count (one: the bf16 h of
    // the mat-0 waves) -- straight-line MFMA code in each (a run-time branch
    // between the two forms inside the loop made the compiler spill ~2.6 k
    // VGPRs)
    auto run = [&](auto nbp_c) __attribute__((always_inline)) {
        constexpr int NB = decltype(nbp_c)::value;
        const LB16 *lb = mat ? la : lh;
        for (int c0 = rb; c0 < re; c0 += WG_BM) {
            __syncthreads();  // the previous chunk's MFMAs are done with LDS
            cz.template store_parts<3>(zi, zi + WG_BM * X3Z, zi + 2 * WG_BM * X3Z, X3Z, yscale, Fo - n0);
            ch.template store_parts<NPH>(hi, hi + WG_BM * X3H, hi + 2 * WG_BM * X3H, X3H, 1.0f, K - k0);
            ca.template store_parts<3>(ai, ai + WG_BM * X3H, ai + 2 * WG_BM * X3H, X3H, 1.0f, K - k0);
            __syncthreads();
            const int c1 = c0 + WG_BM;
            if (c1 < re) {  // the next chunk's loads overlap this chunk's MFMAs
                cz.load(dy, ldy, y, ldyy, nullptr, c1, re, n0, Fo);
                ch.load(h, ldh, nullptr, 0, nullptr, c1, re, k0, K, h_idx, h_rows);
                ca.load(agg, ld_agg, nullptr, 0, rowptr, c1, re, k0, K);
            }
            const int nsteps = re - c0 > 32 ? 2 : 1;  // 32-row MFMA steps holding rows (uniform)
            for (int ks = 0; ks < nsteps; ++ks) {
                const int ro = 32 * ks;
                // Fo tiles NFW w4 + f of the workgroup's 4 NFW
                b8w a1[NFW], a2[NFW], a3[NFW];
#pragma unroll
                for (int f = 0; f < NFW; ++f) {
                    const int c = 16 * (NFW * w4 + f);
                    a1[f] = x3_frag(lz + ro * X3Z, X3Z, c, ln);
                    a2[f] = x3_frag(lz + (WG_BM + ro) * X3Z, X3Z, c, ln);
                    a3[f] = x3_frag(lz + (2 * WG_BM + ro) * X3Z, X3Z, c, ln);
                    if (do_bias) {
                        accb[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a3[f], ones, accb[f], 0, 0, 0);
                        accb[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2[f], ones, accb[f], 0, 0, 0);
                        accb[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[f], ones, accb[f], 0, 0, 0);
                    }
                }
#pragma unroll
                for (int kt = 0; kt < 8; ++kt) {
                    if (kt < KT) {
                        const b8w b1 = x3_frag(lb + ro * X3H, X3H, 16 * kt, ln);
                        b8w b2, b3;
                        if constexpr (NB == 3) {
                            b2 = x3_frag(lb + (WG_BM + ro) * X3H, X3H, 16 * kt, ln);
                            b3 = x3_frag(lb + (2 * WG_BM + ro) * X3H, X3H, 16 * kt, ln);
                        }
#pragma unroll
                        for (int f = 0; f < NFW; ++f) {
                            v4f t = acc[f][kt];
                            if constexpr (NB == 1) {
                                t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a3[f], b1, t, 0, 0, 0);
                                t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2[f], b1, t, 0, 0, 0);
                            } else {
                                t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a3[f], b1, t, 0, 0, 0);
                                t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[f], b3, t, 0, 0, 0);
                                t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2[f], b2, t, 0, 0, 0);
                                t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2[f], b1, t, 0, 0, 0);
                                t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[f], b2, t, 0, 0, 0);
                            }
                            acc[f][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[f], b1, t, 0, 0, 0);
                        }
                    }
                }
            }
        }
    };
    if (HB && mat == 0) run(std::integral_constant<int, 1>{});
    else run(std::integral_constant<int, 3>{});
    // ---- partial slab [Pr Fo x K][Pl Fo x K][Pb Fo] (k_wgrad_partial's layout)
    float *slab = ws + static_cast<size_t>(s) * slab_floats(Fo, K);
    const i32x4 prs = make_rsrc(slab + static_cast<size_t>(mat) * Fo * K,
                                static_cast<uint32_t>(Fo) * static_cast<uint32_t>(K) * 4u);
    const int i16 = ln & 15, q = ln >> 4;
#pragma unroll
    for (int f = 0; f < NFW; ++f)
#pragma unroll
        for (int kt = 0; kt < 8; ++kt) {
            const int k = k0 + 16 * kt + i16;
            const bool kok = k < K && kt < KT;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int n = n0 + 16 * (NFW * w4 + f) + 4 * q + j;
                buf_store1(acc[f][kt][j], prs, (kok && n < n0 + nc) ? (n * K + k) * 4 : kBufOOB, 0, 0);
            }
        }
    if (do_bias && i16 == 0) {
#pragma unroll
        for (int f = 0; f < NFW; ++f)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int n = 16 * (NFW * w4 + f) + 4 * q + j;
                if (n < nc) slab[2 * static_cast<size_t>(Fo) * K + n0 + n] = accb[f][j];
            }
    }
}

// out[i] = sum over the used slabs of slab[s][i], in slab order
__global__ __launch_bounds__(256) void k_wgrad_reduce(const float *__restrict__ ws,
                                                      const int32_t *__restrict__ r_ptr, int S,
                                                      int Fo, int K, float *__restrict__ dwr,
                                                      float *__restrict__ dwl,
                                                      float *__restrict__ db) {
    const int64_t total = slab_floats(Fo, K);
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int used = wgrad_slices(*r_ptr, S);
    // loads issued 32 (then 8) at a time (memory-level parallelism: one HBM
    // round trip per batch), summed in slab order
    float t = 0.0f;
    int s = 0;
    for (; s + 32 <= used; s += 32) {
        float v[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) v[u] = ws[static_cast<size_t>(s + u) * total + i];
#pragma unroll
        for (int u = 0; u < 32; ++u) t += v[u];
    }
    for (; s + 8 <= used; s += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = ws[static_cast<size_t>(s + u) * total + i];
#pragma unroll
        for (int u = 0; u < 8; ++u) t += v[u];
    }
    for (; s < used; ++s) t += ws[static_cast<size_t>(s) * total + i];
    const int64_t FK = static_cast<int64_t>(Fo) * K;
    if (i < FK) dwr[i] = t;
    else if (i < 2 * FK) dwl[i - FK] = t;
    else db[i - 2 * FK] = t;
}

// ---- gather: dh[j] = [j<R] droot[j] + sum_{e in T(j), d=col_t[e] < R} f(dagg[d])
template <int VEC>
struct V;
template <>
struct V<4> {
    using T = float4;
};
template <>
struct V<1> {
    using T = float;
};

template <int VEC>
__device__ __forceinline__ float &cmp(typename V<VEC>::T &v, int i) {
    return reinterpret_cast<float *>(&v)[i];
}

template <int VEC>
__device__ __forceinline__ typename V<VEC>::T ldv(const float *p) {
    return *reinterpret_cast<const typename V<VEC>::T *>(p);
}

template <int VEC, int LPR, int RED>
__global__ __launch_bounds__(256) void k_dgrad_gather(
    const float *__restrict__ dagg, int64_t ld_dagg, const float *__restrict__ droot,
    int64_t ld_droot, const int32_t *__restrict__ rowptr, const int32_t *__restrict__ rowptr_t,
    const int32_t *__restrict__ col_t, int n_rows, const int32_t *__restrict__ r_ptr,
    const int32_t *__restrict__ rn_ptr, int K, const float *__restrict__ h, int64_t ldh,
    const float *__restrict__ agg, int64_t ld_agg, float *__restrict__ dh, int64_t ldd,
    int zero_tail) {
    using T = typename V<VEC>::T;
    constexpr int GROUPS = 256 / LPR;
    const int lane = threadIdx.x % LPR;
    const int64_t row = (int64_t)blockIdx.x * GROUPS + threadIdx.x / LPR;
    if (row >= n_rows) return;
    const int R = *r_ptr, Rn = *rn_ptr;
    const int nchunks = (K + LPR * VEC - 1) / (LPR * VEC);
    if (row >= Rn) {
        if (zero_tail)
            for (int ch = 0; ch < nchunks; ++ch) {
                const int f = ch * LPR * VEC + lane * VEC;
                if (f < K) {
                    T z;
#pragma unroll
                    for (int i = 0; i < VEC; ++i) cmp<VEC>(z, i) = 0.0f;
                    *reinterpret_cast<T *>(dh + row * ldd + f) = z;
                }
            }
        return;
    }
    const int beg = rowptr_t[row], end = rowptr_t[row + 1];
    for (int ch = 0; ch < nchunks; ++ch) {
        const int f = ch * LPR * VEC + lane * VEC;
        const bool act = f < K;
        T acc, xv;
#pragma unroll
        for (int i = 0; i < VEC; ++i) cmp<VEC>(acc, i) = 0.0f;
        if (RED == NGNN_REDUCE_MAX && act) xv = ldv<VEC>(h + row * ldh + f);
        for (int eb = beg; eb < end; eb += LPR) {
            const int n = min(LPR, end - eb);
            int myd = 0x7fffffff;
            float myc = 1.0f;
            if (lane < n) {
                myd = col_t[eb + lane];
                if (RED == NGNN_REDUCE_MEAN && myd < R) {
                    const int dg = rowptr[myd + 1] - rowptr[myd];
                    myc = static_cast<float>(dg > 1 ? dg : 1);
                }
            }
            for (int k = 0; k < n; ++k) {
                const int d = __shfl(myd, k, LPR);
                const float cn = __shfl(myc, k, LPR);
                if (d >= R || !act) continue;  // edge into a row whose gradient is zero
                const T g = ldv<VEC>(dagg + static_cast<int64_t>(d) * ld_dagg + f);
                if (RED == NGNN_REDUCE_MAX) {
                    const T av = ldv<VEC>(agg + static_cast<int64_t>(d) * ld_agg + f);
#pragma unroll
                    for (int i = 0; i < VEC; ++i) {
                        const float m = (cmp<VEC>(xv, i) == reinterpret_cast<const float *>(&av)[i]) ? 1.0f : 0.0f;
                        cmp<VEC>(acc, i) += m * reinterpret_cast<const float *>(&g)[i];
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < VEC; ++i) {
                        const float t = reinterpret_cast<const float *>(&g)[i];
                        cmp<VEC>(acc, i) += (RED == NGNN_REDUCE_MEAN) ? t / cn : t;
                    }
                }
            }
        }
        if (!act) continue;
        if (row < R) {
            const T rt = ldv<VEC>(droot + row * ld_droot + f);
#pragma unroll
            for (int i = 0; i < VEC; ++i)
                cmp<VEC>(acc, i) = reinterpret_cast<const float *>(&rt)[i] + cmp<VEC>(acc, i);
        }
        *reinterpret_cast<T *>(dh + row * ldd + f) = acc;
    }
}

// MAX: gdist[d] = dagg[d] / ([agg[d]==0] + #{e into d: h[src_e]==agg[d]}),  d < R
template <int VEC, int LPR>
__global__ __launch_bounds__(256) void k_max_gdist(const float *__restrict__ dagg, int64_t ld_dagg,
                                                   const int32_t *__restrict__ rowptr,
                                                   const int32_t *__restrict__ col, int n_rows,
                                                   const int32_t *__restrict__ r_ptr, int K,
                                                   const float *__restrict__ h, int64_t ldh,
                                                   const float *__restrict__ agg, int64_t ld_agg,
                                                   float *__restrict__ gdist) {
    using T = typename V<VEC>::T;
    constexpr int GROUPS = 256 / LPR;
    const int lane = threadIdx.x % LPR;
    const int64_t row = (int64_t)blockIdx.x * GROUPS + threadIdx.x / LPR;
    if (row >= n_rows || row >= *r_ptr) return;
    const int beg = rowptr[row], end = rowptr[row + 1];
    if (beg == end) return;  // never referenced by the gather
    const int nchunks = (K + LPR * VEC - 1) / (LPR * VEC);
    for (int ch = 0; ch < nchunks; ++ch) {
        const int f = ch * LPR * VEC + lane * VEC;
        const bool act = f < K;
        T a, ties;
        if (act) a = ldv<VEC>(agg + row * ld_agg + f);
#pragma unroll
        for (int i = 0; i < VEC; ++i)
            cmp<VEC>(ties, i) = (act && cmp<VEC>(a, i) == 0.0f) ? 1.0f : 0.0f;
        for (int eb = beg; eb < end; eb += LPR) {
            const int n = min(LPR, end - eb);
            const int myc = lane < n ? col[eb + lane] : 0;
            for (int k = 0; k < n; ++k) {
                const int c = __shfl(myc, k, LPR);
                if (!act) continue;
                const T v = ldv<VEC>(h + static_cast<int64_t>(c) * ldh + f);
#pragma unroll
                for (int i = 0; i < VEC; ++i)
                    cmp<VEC>(ties, i) += (reinterpret_cast<const float *>(&v)[i] == cmp<VEC>(a, i)) ? 1.0f : 0.0f;
            }
        }
        if (!act) continue;
        T g = ldv<VEC>(dagg + row * ld_dagg + f);
#pragma unroll
        for (int i = 0; i < VEC; ++i) cmp<VEC>(g, i) = cmp<VEC>(g, i) / cmp<VEC>(ties, i);
        *reinterpret_cast<T *>(gdist + row * static_cast<int64_t>(K) + f) = g;
    }
}

// ---- atomic path (default; like the reference's CUDA index_add_ backward)
// dh[j] = [j < R] droot[j] for j < Rn; rows >= Rn zeroed if zero_tail
// VEC (K, ldd, ld_droot multiples of 4, 16-B aligned rows): 16-B stores,
// and when K / 4 divides 256 each thread keeps one column quad (no division
// in the loop) -- a zero fill of ~340 MB per step in the 3-layer config
template <bool VEC>
__global__ __launch_bounds__(256) void k_dh_init(const float *__restrict__ droot, int64_t ld_droot,
                                                 int n_rows, const int32_t *__restrict__ r_ptr,
                                                 const int32_t *__restrict__ rn_ptr, int K,
                                                 float *__restrict__ dh, int64_t ldd, int zero_tail) {
    const int R = *r_ptr, Rn = *rn_ptr;
    const int64_t lim = zero_tail ? n_rows : min(n_rows, Rn);
    const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
    const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (VEC) {
        const int K4 = K >> 2;
        if (256 % K4 == 0) {
            const int f = 4 * static_cast<int>(threadIdx.x % K4);
            const int64_t rstep = nthr / K4;
            for (int64_t row = tid / K4; row < lim; row += rstep) {
                v4f v{0.f, 0.f, 0.f, 0.f};
                if (droot && row < R) v = *reinterpret_cast<const v4f *>(droot + row * ld_droot + f);
                *reinterpret_cast<v4f *>(dh + row * ldd + f) = v;
            }
        } else {
            for (int64_t idx = tid; idx < lim * K4; idx += nthr) {
                const int64_t row = idx / K4;
                const int f = 4 * static_cast<int>(idx - row * K4);
                v4f v{0.f, 0.f, 0.f, 0.f};
                if (droot && row < R) v = *reinterpret_cast<const v4f *>(droot + row * ld_droot + f);
                *reinterpret_cast<v4f *>(dh + row * ldd + f) = v;
            }
        }
        return;
    }
    for (int64_t idx = tid; idx < lim * K; idx += nthr) {
        const int64_t row = idx / K;
        const int f = static_cast<int>(idx - row * K);
        dh[row * ldd + f] = (droot && row < R) ? droot[row * ld_droot + f] : 0.0f;
    }
}

void dh_init_launch(const float *droot, int64_t ld_droot, int64_t n_rows, const int32_t *r_ptr,
                    const int32_t *rn_ptr, int64_t K, float *dh, int64_t ldd, int zero_tail, hipStream_t st) {
    const bool vec = K % 4 == 0 && ldd % 4 == 0 && aligned(dh, 16) &&
                     (!droot || (ld_droot % 4 == 0 && aligned(droot, 16)));
    const unsigned g = static_cast<unsigned>(std::min<int64_t>(ceil_div(n_rows * K, vec ? 1024 : 256), 4096));
    if (vec)
        hipLaunchKernelGGL(k_dh_init<true>, dim3(std::max(g, 1u)), dim3(256), 0, st, droot, ld_droot, (int)n_rows,
                           r_ptr, rn_ptr, (int)K, dh, ldd, zero_tail);
    else
        hipLaunchKernelGGL(k_dh_init<false>, dim3(std::max(g, 1u)), dim3(256), 0, st, droot, ld_droot, (int)n_rows,
                           r_ptr, rn_ptr, (int)K, dh, ldd, zero_tail);
}

// one wave per target row d < R: scale dagg[d] once, then one 256-B atomic
// wave-instruction per (in-edge, 64 columns) into the source row
template <int RED>
__global__ __launch_bounds__(256) void k_dgrad_scatter(
    const float *__restrict__ dagg, int64_t ld_dagg, const int32_t *__restrict__ rowptr,
    const int32_t *__restrict__ col, int n_rows, const int32_t *__restrict__ r_ptr, int K,
    const float *__restrict__ h, int64_t ldh, const float *__restrict__ agg, int64_t ld_agg,
    float *__restrict__ dh, int64_t ldd) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int R = min(n_rows, *r_ptr);
    for (int64_t d = blockIdx.x * 4 + wave; d < R; d += gridDim.x * 4) {
        const int beg = rowptr[d], end = rowptr[d + 1];
        if (beg == end) continue;
        const float cnt = static_cast<float>(end - beg);
        for (int f0 = 0; f0 < K; f0 += 64) {
            const int f = f0 + lane;
            const bool act = f < K;
            float v = act ? dagg[d * ld_dagg + f] : 0.0f;
            float a = 0.0f;
            if (RED == NGNN_REDUCE_MEAN) v = v / cnt;
            if (RED == NGNN_REDUCE_MAX) {
                a = act ? agg[d * ld_agg + f] : 0.0f;
                float ties = (a == 0.0f) ? 1.0f : 0.0f;
                for (int e = beg; e < end; ++e) {
                    const int64_t j = col[e];
                    if (act) ties += (h[j * ldh + f] == a) ? 1.0f : 0.0f;
                }
                v = v / ties;
            }
            if (!act) continue;
            for (int e = beg; e < end; ++e) {
                const int64_t j = col[e];
                if (RED == NGNN_REDUCE_MAX && !(h[j * ldh + f] == a)) continue;
                atomicAdd(dh + j * ldd + f, v);
            }
        }
    }
}

// ---- fused dgrad (atomic): no dgrad GEMM launch.  One wave per target row
// d < R (grid-stride, so rows past the device-side bound cost nothing):
//   dz[d]    = dy[d] (* [y > 0] * yscale)            staged in the wave's LDS slot
//   root[f]  = sum_n dz[d][n] W_r[n][f]   -> atomic into dh[d][f]
//   agg[f]   = sum_n dz[d][n] W_l[n][f]   -> scaled (mean: / deg; max: tie split)
//              and atomically added into dh[j][f] for every in-edge j -> d
// lanes own 64 consecutive columns per chunk, so every atomic wave-instruction
// covers 256 contiguous bytes; W rows are read coalesced from L1/L2.
// dh rows < Rn must be zeroed first (k_dh_init with droot = NULL semantics).
constexpr int FD_MAXF = 512;  // dz row staged per wave: Fo <= 512 on this path

// LDS_W: W_r and W_l ([Fo][K] each, row-major as given) are first copied into
// LDS by the (persistent) workgroup, so the per-row products read LDS
// (~64-cycle latency, conflict-free: lanes read consecutive columns) instead
// of chains of L2 loads.  Dynamic LDS: 2 Fo K floats.
template <int RED, bool LDS_W>
__global__ __launch_bounds__(256) void k_dgrad_fused(
    const float *__restrict__ dy, int64_t ldy, const float *__restrict__ y, int64_t ldyy,
    float yscale, const float *__restrict__ wl_g, const float *__restrict__ wr_g, int Fo, int K,
    const int32_t *__restrict__ rowptr, const int32_t *__restrict__ col, int n_rows,
    const int32_t *__restrict__ r_ptr, const float *__restrict__ h, int64_t ldh,
    const float *__restrict__ agg, int64_t ld_agg, float *__restrict__ dh, int64_t ldd) {
    __shared__ __attribute__((aligned(16))) float sdz[4][FD_MAXF];
    extern __shared__ __attribute__((aligned(16))) float sw[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float *z = sdz[wave];
    const int R = min(n_rows, *r_ptr);
    // work item = (target row d, 64-column chunk): a few hundred seed rows
    // still fill the chip (one wave per row ran the 512-wide chunks of
    // Amazon-Computers' hidden layer back to back: 80 us for 300 rows)
    const int nch = (K + 63) >> 6;
    const int64_t items = static_cast<int64_t>(R) * nch;
    const float *wr = wr_g, *wl = wl_g;
    if (LDS_W) {
        if (static_cast<int64_t>(blockIdx.x) * 4 >= items) return;  // no work for this workgroup
        const int n4 = (Fo * K) >> 2;  // Fo K % 4 == 0 on this path
        float4 *s4 = reinterpret_cast<float4 *>(sw);
        const float4 *r4 = reinterpret_cast<const float4 *>(wr_g);
        const float4 *l4 = reinterpret_cast<const float4 *>(wl_g);
        for (int i = threadIdx.x; i < n4; i += 256) {
            s4[i] = r4[i];
            s4[n4 + i] = l4[i];
        }
        __syncthreads();
        wr = sw;
        wl = sw + Fo * K;
    }
    for (int64_t w = blockIdx.x * 4 + wave; w < items; w += gridDim.x * 4) {
        const int64_t d = w / nch;
        for (int n = lane; n < Fo; n += 64) {
            float v = dy[d * ldy + n];
            if (y) v = (y[d * ldyy + n] > 0.0f) ? v * yscale : 0.0f;
            z[n] = v;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // z[] written by all lanes
        __builtin_amdgcn_wave_barrier();
        const int beg = rowptr[d], end = rowptr[d + 1];
        const float cnt = static_cast<float>(end - beg);
        do {  // (continue: this lane is done with the item)
            const int f0 = static_cast<int>(w - d * nch) * 64;
            const int f = f0 + lane;
            const bool act = f < K;
            const int fc = act ? f : 0;
            float ar = 0.0f, al = 0.0f;
            int n = 0;
            for (; n + 4 <= Fo; n += 4) {
                const float4 zz = *reinterpret_cast<const float4 *>(z + n);  // uniform: broadcast
                const float r0 = wr[(int64_t)(n + 0) * K + fc], r1 = wr[(int64_t)(n + 1) * K + fc];
                const float r2 = wr[(int64_t)(n + 2) * K + fc], r3 = wr[(int64_t)(n + 3) * K + fc];
                const float l0 = wl[(int64_t)(n + 0) * K + fc], l1 = wl[(int64_t)(n + 1) * K + fc];
                const float l2 = wl[(int64_t)(n + 2) * K + fc], l3 = wl[(int64_t)(n + 3) * K + fc];
                ar += zz.x * r0; ar += zz.y * r1; ar += zz.z * r2; ar += zz.w * r3;
                al += zz.x * l0; al += zz.y * l1; al += zz.z * l2; al += zz.w * l3;
            }
            for (; n < Fo; ++n) {
                const float zn = z[n];
                ar += zn * wr[(int64_t)n * K + fc];
                al += zn * wl[(int64_t)n * K + fc];
            }
            if (!act) continue;
            atomicAdd(dh + d * ldd + f, ar);
            if (beg == end) continue;
            float v = al;
            float a = 0.0f;
            if (RED == NGNN_REDUCE_MEAN) v = v / cnt;
            if (RED == NGNN_REDUCE_MAX) {
                a = agg[d * ld_agg + f];
                float ties = (a == 0.0f) ? 1.0f : 0.0f;
                for (int e = beg; e < end; ++e) ties += (h[(int64_t)col[e] * ldh + f] == a) ? 1.0f : 0.0f;
                v = v / ties;
            }
            for (int e = beg; e < end; ++e) {
                const int64_t j = col[e];
                if (RED == NGNN_REDUCE_MAX && !(h[j * ldh + f] == a)) continue;
                atomicAdd(dh + j * ldd + f, v);
            }
        } while (0);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // done reading z
        __builtin_amdgcn_wave_barrier();
    }
}

// ---- low-dimensional input gradient (MEAN/SUM, Fo < K).  The aggregation
// is linear, so  sum_{d <- j} (dz[d] W_l) / deg(d) = (sum_{d <- j} dz[d] /
// deg(d)) W_l : scatter dz in the Fo-wide space first, then ONE dense MFMA
// pass  dh[j] = [j < R] dz[j] W_r + g[j] W_l  over rows < Rn.  For the
// products output layer (Fo = 47, K = 256) that is 5.4x fewer atomics and no
// zero-fill of dh (every row < Rn is written once).
//
// ws = [W image | g]: the image ([KS][NTP][64] floats, MFMA A-operand order:
// element (ks, t, lane = (i16, kk)) = Wcat[4 ks + kk][16 t + i16], Wcat =
// [W_r ; W_l] with each half padded to C4 rows) is rebuilt every call by the
// scatter launch's extra workgroups; g = [n_rows][C4] floats (C4 = Fo rounded
// up to 4) is zero on entry and the dense pass clears each row as it reads
// it, so g is zero again on exit.
constexpr int LD_ROWS = 64;
__host__ __device__ inline int64_t lowdim_img_floats(int64_t Fo, int ntp) {
    const int64_t C4 = (Fo + 3) & ~int64_t{3};
    return (C4 / 2) * ntp * 64;
}

template <bool MEAN, bool MASK>
__global__ __launch_bounds__(256) void k_lowdim_scatter(
    const float *__restrict__ dy, int64_t ldy, const float *__restrict__ y, int64_t ldyy,
    float yscale, const int32_t *__restrict__ rowptr, const int32_t *__restrict__ col, int n_rows,
    const int32_t *__restrict__ r_ptr, int Fo, int C4, float *__restrict__ g, int n_scatter_wg,
    const float *__restrict__ wl, const float *__restrict__ wr, int64_t ldw, int K, int ntp,
    float *__restrict__ img) {
    if (static_cast<int>(blockIdx.x) >= n_scatter_wg) {  // W image packing workgroups
        const int64_t idx = (static_cast<int64_t>(blockIdx.x) - n_scatter_wg) * 256 + threadIdx.x;
        if (idx >= lowdim_img_floats(Fo, ntp)) return;
        const int ln = static_cast<int>(idx & 63);
        const int t = static_cast<int>((idx >> 6) % ntp), ks = static_cast<int>(idx / (64 * ntp));
        const int n = t * 16 + (ln & 15), i = ks * 4 + (ln >> 4);
        float v = 0.0f;
        if (n < K) {
            if (i < C4) {
                if (i < Fo) v = wr[static_cast<int64_t>(i) * ldw + n];
            } else if (i - C4 < Fo) {
                v = wl[static_cast<int64_t>(i - C4) * ldw + n];
            }
        }
        img[idx] = v;
        return;
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int R = min(n_rows, *r_ptr);
    for (int64_t d = blockIdx.x * 4 + wave; d < R; d += n_scatter_wg * 4) {
        const int beg = rowptr[d], end = rowptr[d + 1];
        if (beg == end) continue;
        const float inv = MEAN ? 1.0f / static_cast<float>(end - beg) : 1.0f;
        for (int f0 = 0; f0 < Fo; f0 += 64) {
            const int f = f0 + lane;
            float v = 0.0f;
            if (f < Fo) {
                v = dy[d * ldy + f];
                if (MASK) v = (y[d * ldyy + f] > 0.0f) ? v * yscale : 0.0f;
                if (MEAN) v *= inv;
            }
            // sources preloaded 64 at a time and broadcast, so the atomics of
            // one row issue back to back (no index load between them)
            for (int eb = beg; eb < end; eb += 64) {
                const int ne = min(64, end - eb);
                const int mycol = lane < ne ? col[eb + lane] : 0;
                for (int k = 0; k < ne; ++k) {
                    const int64_t j = __shfl(mycol, k);
                    if (f < Fo && v != 0.0f) atomicAdd(g + j * C4 + f, v);  // exact 0 adds nothing
                }
            }
        }
    }
}

// dense pass.  Workgroup (512 threads) = an even share [rb, re) of rows < Rn
// on 16-row boundaries, staged 64 rows at a time as X = [dz | g] ([64][2 C4],
// dz rows >= R and g rows >= Rn read as 0); the W image is copied to LDS once.
// Wave w: row tile w >> 1, column half w & 1 (NTW tiles); a lane's
// accumulator holds 4 consecutive output columns of one row -> 16-B stores.
constexpr int LD_SU = 8;  // loads in flight per thread per staging batch
template <int NTW, bool VOUT>
__global__ __launch_bounds__(512, 1) void k_lowdim_gemm(
    const float *__restrict__ dy, int64_t ldy, const float *__restrict__ y, int64_t ldyy,
    float yscale, const float *__restrict__ img, int Fo, int K, int n_rows,
    const int32_t *__restrict__ r_ptr, const int32_t *__restrict__ rn_ptr, float *__restrict__ g,
    int C4, float *__restrict__ dh, int64_t ldd) {
    extern __shared__ __attribute__((aligned(16))) float lsm[];
    constexpr int NTP = 2 * NTW;         // tiles in the image (K <= 16 NTP)
    const int KS = C4 / 2;               // k-steps: 2 C4 / 4
    const int LDX = 2 * C4 + 4;          // staged row stride (floats)
    float *wimg = lsm;                   // [KS][NTP][64]
    float *xs = lsm + KS * NTP * 64;     // [64][LDX]
    const int R = min(n_rows, *r_ptr);
    const int Rn = min(n_rows, *rn_ptr);
    const int T16 = (Rn + 15) >> 4;      // 16-row tiles below Rn
    const int G = gridDim.x;
    const int rb = 16 * static_cast<int>(static_cast<int64_t>(blockIdx.x) * T16 / G);
    const int re = min(Rn, 16 * static_cast<int>(static_cast<int64_t>(blockIdx.x + 1) * T16 / G));
    if (rb >= re) return;
    {  // W image -> LDS, 2 LD_SU 16-B loads in flight per thread (the
       // products output layer's 96 KiB image: one batch)
        const int n4 = KS * NTP * 16;
        const v4f *src = reinterpret_cast<const v4f *>(img);
        v4f *dst = reinterpret_cast<v4f *>(wimg);
        constexpr int IU = 2 * LD_SU;
        for (int base = 0; base < n4; base += 512 * IU) {
            v4f t[IU];
#pragma unroll
            for (int u = 0; u < IU; ++u) {
                const int i = base + u * 512 + threadIdx.x;
                if (i < n4) t[u] = src[i];
            }
#pragma unroll
            for (int u = 0; u < IU; ++u) {
                const int i = base + u * 512 + threadIdx.x;
                if (i < n4) dst[i] = t[u];
            }
        }
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int rt = wave >> 1, chf = wave & 1;
    const int i16 = lane & 15, kk = lane >> 4;
    const int C44 = C4 >> 2;
    for (int c0 = rb; c0 < re; c0 += LD_ROWS) {
        __syncthreads();  // W image written / previous stage's reads done
        const int nr = min(LD_ROWS, re - c0);
        // dz half (scalar: Fo need not be a multiple of 4; rows < R only)
        // and g half (16-B loads, each read row cleared behind it), one
        // batch of each: every load of the stage is in flight before the
        // first LDS store (C4 <= 64: 64 C4 <= 512 LD_SU)
        auto ld_dz = [&](int base, float (&t)[LD_SU]) {
#pragma unroll
            for (int u = 0; u < LD_SU; ++u) {
                const int idx = base + u * 512 + threadIdx.x;
                const int r = idx / C4, c = idx - r * C4;
                const int64_t j = c0 + r;
                t[u] = 0.0f;
                if (r < nr && c < Fo && j < R) {
                    float v = dy[j * ldy + c];
                    if (y) v = (y[j * ldyy + c] > 0.0f) ? v * yscale : 0.0f;
                    t[u] = v;
                }
            }
        };
        auto st_dz = [&](int base, const float (&t)[LD_SU]) {
#pragma unroll
            for (int u = 0; u < LD_SU; ++u) {
                const int idx = base + u * 512 + threadIdx.x;
                const int r = idx / C4, c = idx - r * C4;
                if (r < LD_ROWS) xs[r * LDX + c] = t[u];
            }
        };
        auto ld_g = [&](int base, v4f (&t)[LD_SU]) {
#pragma unroll
            for (int u = 0; u < LD_SU; ++u) {
                const int idx = base + u * 512 + threadIdx.x;
                const int r = idx / C44, c = (idx - r * C44) * 4;
                t[u] = v4f{0.f, 0.f, 0.f, 0.f};
                if (r < nr) {
                    v4f *gp = reinterpret_cast<v4f *>(g + (c0 + r) * static_cast<int64_t>(C4) + c);
                    t[u] = *gp;
                    *gp = v4f{0.f, 0.f, 0.f, 0.f};  // leave g zero for the next call
                }
            }
        };
        auto st_g = [&](int base, const v4f (&t)[LD_SU]) {
#pragma unroll
            for (int u = 0; u < LD_SU; ++u) {
                const int idx = base + u * 512 + threadIdx.x;
                const int r = idx / C44, c = (idx - r * C44) * 4;
                if (r < LD_ROWS) *reinterpret_cast<v4f *>(xs + r * LDX + C4 + c) = t[u];
            }
        };
        if (LD_ROWS * C4 <= 512 * LD_SU) {
            float tz[LD_SU];
            v4f tg[LD_SU];
            ld_dz(0, tz);
            ld_g(0, tg);
            st_dz(0, tz);
            st_g(0, tg);
        } else {
            for (int base = 0; base < LD_ROWS * C4; base += 512 * LD_SU) {
                float t[LD_SU];
                ld_dz(base, t);
                st_dz(base, t);
            }
            for (int base = 0; base < LD_ROWS * C44; base += 512 * LD_SU) {
                v4f t[LD_SU];
                ld_g(base, t);
                st_g(base, t);
            }
        }
        __syncthreads();
        if (rt * 16 >= nr) continue;  // this wave's row tile is past the stage
        v4f acc[NTW];
#pragma unroll
        for (int t = 0; t < NTW; ++t) acc[t] = v4f{0.f, 0.f, 0.f, 0.f};
        const float *xb = xs + (rt * 16 + i16) * LDX + kk;
        const float *wb = wimg + chf * NTW * 64 + lane;
        float b = xb[0], a[NTW];
#pragma unroll
        for (int t = 0; t < NTW; ++t) a[t] = wb[t * 64];
        for (int ks = 0; ks < KS; ++ks) {  // LDS reads of ks+1 before the MFMAs of ks
            const int kn = min(ks + 1, KS - 1);
            const float bn = xb[kn * 4];
            float an[NTW];
#pragma unroll
            for (int t = 0; t < NTW; ++t) an[t] = wb[(kn * NTP + t) * 64];
#pragma unroll
            for (int t = 0; t < NTW; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], b, acc[t], 0, 0, 0);
            b = bn;
#pragma unroll
            for (int t = 0; t < NTW; ++t) a[t] = an[t];
        }
        const int64_t row = c0 + rt * 16 + i16;
        if (row < re) {
#pragma unroll
            for (int t = 0; t < NTW; ++t) {
                const int f = (chf * NTW + t) * 16 + 4 * kk;
                float *o = dh + row * ldd + f;
                if (VOUT) {
                    if (f < K) *reinterpret_cast<v4f *>(o) = acc[t];
                } else {
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj)
                        if (f + jj < K) o[jj] = acc[t][jj];
                }
            }
        }
    }
}

int lpr_for(int64_t K, int vec) {
    const int64_t chunks = ceil_div(K, vec);
    int l = 4;
    while (l < 64 && l < chunks) l <<= 1;
    return l;
}

}  // namespace
}  // namespace ngnn

using namespace ngnn;

extern "C" size_t ngnn_sage_wgrad_workspace_bytes(int64_t Fo, int64_t K) {
    if (Fo <= 0 || K <= 0) return 0;
    return sizeof(float) * S_MAX * slab_floats(Fo, K);
}

template <int NTW, int KTW, bool SPLIT_N>
static void launch_wgrad(dim3 grid, hipStream_t st, bool vz, int vh, const float *dy, int64_t ldy,
                         const float *y, int64_t ldyy, bool y_bf16, float yscale, const float *h,
                         const float *const *h_dev, int64_t ldh, const int64_t *h_idx,
                         const int64_t *const *h_idx_dev, int64_t h_rows, const float *agg,
                         int64_t ld_agg, const int32_t *rowptr, const int32_t *r_ptr, int Fo, int K,
                         float *ws) {
    auto go = [&](auto vz_c, auto vh_c, auto m_c) {
        hipLaunchKernelGGL((k_wgrad_partial<NTW, KTW, SPLIT_N, decltype(vz_c)::value,
                                            decltype(vh_c)::value, decltype(m_c)::value>),
                           grid, dim3(512), 0, st, dy, ldy, y, ldyy, yscale, h, h_dev, ldh, h_idx,
                           h_idx_dev, h_rows, agg, ld_agg, rowptr, r_ptr, Fo, K, ws);
    };
    using T = std::true_type;
    using F = std::false_type;
    auto with_mask = [&](auto vz_c, auto vh_c) {
        if (y && y_bf16) go(vz_c, vh_c, std::integral_constant<int, 2>{});
        else if (y) go(vz_c, vh_c, std::integral_constant<int, 1>{});
        else go(vz_c, vh_c, std::integral_constant<int, 0>{});
    };
    using V0 = std::integral_constant<int, 0>;
    using V1 = std::integral_constant<int, 1>;
    using V2 = std::integral_constant<int, 2>;
    if (vz) {
        if (vh == 2) with_mask(T{}, V2{});
        else if (vh) with_mask(T{}, V1{});
        else with_mask(T{}, V0{});
    } else {
        if (vh == 2) with_mask(F{}, V2{});
        else if (vh) with_mask(F{}, V1{});
        else with_mask(F{}, V0{});
    }
}

extern "C" int ngnn_sage_wgrad(const float *dy, int64_t ldy, const float *y, int64_t ldyy,
                               float yscale, const float *h, const float *const *h_dev,
                               const int64_t *h_idx, const int64_t *const *h_idx_dev, int64_t h_rows,
                               int bf16_flags, int64_t ldh, const float *agg, int64_t ld_agg,
                               const int32_t *rowptr, int64_t n_rows, const int32_t *r_ptr,
                               int64_t Fo, int64_t K, float *dwl, float *dbl, float *dwr, void *ws,
                               size_t ws_bytes, void *stream) {
    NGNN_RETURN_IF(!dy || (!h && !h_dev) || !agg || !rowptr || !r_ptr || !dwl || !dbl || !dwr,
                   NGNN_E_ARG);
    NGNN_RETURN_IF(Fo <= 0 || K <= 0 || n_rows < 0, NGNN_E_ARG);
    NGNN_RETURN_IF(ldy < Fo || ldh < K || ld_agg < K || (y && ldyy < Fo), NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(n_rows) || !fits_i32(K), NGNN_E_RANGE);
    // 32-bit buffer offsets: a 64-row chunk of every operand and one partial
    // matrix must stay below 2 GiB
    NGNN_RETURN_IF(ldy > (1 << 22) || ldh > (1 << 22) || ld_agg > (1 << 22) ||
                   (y && ldyy > (1 << 22)) || Fo * K > (int64_t{1} << 28), NGNN_E_RANGE);
    NGNN_RETURN_IF(!ws || ws_bytes < ngnn_sage_wgrad_workspace_bytes(Fo, K), NGNN_E_WORKSPACE);
    // bf16_flags: 1 h rows bf16, 2 mask rows y bf16
    const int h_bf16 = bf16_flags & 1;
    const bool y_bf16 = (bf16_flags & 2) != 0;
    // indexed h (the feature table under the fused x[n_id] gather): 32-bit
    // offsets over the whole table
    NGNN_RETURN_IF((h_idx || h_idx_dev) && (h_rows <= 0 || h_rows * ldh * 4 >= (int64_t{1} << 31)),
                   NGNN_E_RANGE);
    // bf16 h (a bf16 model's layer input): 8-B loads, rows 8-B aligned
    NGNN_RETURN_IF(h_bf16 && (K % 4 != 0 || ldh % 4 != 0 || ld_agg % 4 != 0 ||
                              (!h_dev && !aligned(h, 8)) || !aligned(agg, 16)),
                   NGNN_E_SHAPE);
    // 16-B staging per operand pair: dz (+ its mask y) and h / agg
    const bool vz = (Fo % 4 == 0) && (ldy % 4 == 0) && aligned(dy, 16) &&
                    (!y || ((ldyy % 4 == 0) && aligned(y, y_bf16 ? 8 : 16)));
    const int vh = h_bf16 ? 2
                          : ((K % 4 == 0) && (ldh % 4 == 0) && (ld_agg % 4 == 0) &&
                             (h_dev || aligned(h, 16)) && aligned(agg, 16));  // h_dev: 16-B aligned by contract
    hipStream_t st = as_stream(stream);
    float *wsf = static_cast<float *>(ws);
    // slices x K-chunks x Fo-chunks ~ one workgroup per CU; the kernel uses
    // min(S, R/64) slices for the device-side row bound R
    const int64_t gy = ceil_div(K, WG_KC), gz = ceil_div(Fo, WG_NC);
    const int S = static_cast<int>(std::max<int64_t>(
        1, std::min<int64_t>(ceil_div(n_rows, WG_BM), std::max<int64_t>(1, S_MAX / (gy * gz)))));
    const dim3 grid(S, static_cast<unsigned>(gy), static_cast<unsigned>(gz));
    const int NT = static_cast<int>(ceil_div(std::min<int64_t>(Fo, WG_NC), 16));
#define NGNN_WG_ARGS grid, st, vz, vh, dy, ldy, y, ldyy, y_bf16, yscale, h, h_dev, ldh, h_idx, h_idx_dev, \
                     h_rows, agg, ld_agg, rowptr, r_ptr, (int)Fo, (int)K, wsf
    // (NGNN_WGRAD_X3=0, read once: the exact-f32 MFMA kernel for every shape -- A/B)
    static const bool x3_on = [] {
        const char *e = std::getenv("NGNN_WGRAD_X3");
        return !(e && e[0] == '0');
    }();
    // (fp32 h / agg rows at 4-B alignment, K % 4 != 0 -- Amazon-Computers' K =
    // 767: the X3 kernel's 16-B loads read past K into the next row, and
    // store_parts zeroes those columns)
    const bool vh_x3 = vh || (!h_bf16 && (h_dev || aligned(h, 4)) && aligned(agg, 4));
    if (NT == 4 && vz && vh_x3 && x3_on) {
        const bool hb = vh == 2;
        // bf16 h with Fo >= 128: two Fo tiles per wave (half the h / agg re-reads)
        // (NGNN_WGRAD_NFW=2, read once: two Fo tiles per wave -- half the
        // h / agg re-reads, but the bf16-mask form spills: 429 vs 250 us on
        // config #3's layer 0, A/B only)
        static const int nfw_max = [] {
            const char *e = std::getenv("NGNN_WGRAD_NFW");
            return e ? std::max(1, std::min(2, std::atoi(e))) : 1;
        }();
        const int nfw = hb && Fo >= 128 ? nfw_max : 1;
        const size_t lds = (static_cast<size_t>(3) * WG_BM * (WG_NC * nfw + 16) + (hb ? 1 : 3) * WG_BM * X3H +
                            static_cast<size_t>(3) * WG_BM * X3H) * 2;
        const int gz2 = static_cast<int>(ceil_div(Fo, WG_NC * nfw));
        const dim3 grid2(static_cast<unsigned>(ceil_div(static_cast<int64_t>(S) * gy, 8) * 8 * gz2));
        auto go = [&](auto hb_c, auto m_c) {
            constexpr bool HBv = decltype(hb_c)::value;
            auto fn = (HBv && nfw == 2) ? k_wgrad_x3<HBv, decltype(m_c)::value, 2>
                                        : k_wgrad_x3<HBv, decltype(m_c)::value, 1>;
            static bool attr[3] = {false, false, false};  // per NFW; benign race: idempotent
            if (!attr[nfw]) {
                (void)hipFuncSetAttribute(reinterpret_cast<const void *>(fn),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                attr[nfw] = true;
            }
            hipLaunchKernelGGL(fn, grid2, dim3(512), lds, st, dy, ldy, y, ldyy, yscale, h, h_dev, ldh,
                               h_idx, h_idx_dev, h_rows, agg, ld_agg, rowptr, r_ptr, (int)Fo, (int)K, wsf, S,
                               static_cast<int>(gy), gz2);
        };
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        using I2 = std::integral_constant<int, 2>;
        auto by_mask = [&](auto hb_c) {
            if (y && y_bf16) go(hb_c, I2{});
            else if (y) go(hb_c, I1{});
            else go(hb_c, I0{});
        };
        if (hb) by_mask(std::true_type{});
        else by_mask(std::false_type{});
    } else if (NT == 4) launch_wgrad<1, 8, true>(NGNN_WG_ARGS);
    else if (NT == 1) launch_wgrad<1, 2, false>(NGNN_WG_ARGS);
    else if (NT == 2) launch_wgrad<2, 2, false>(NGNN_WG_ARGS);
    else launch_wgrad<3, 2, false>(NGNN_WG_ARGS);
#undef NGNN_WG_ARGS
    int rc = launch_status();
    if (rc) return rc;
    const int64_t total = static_cast<int64_t>(slab_floats(Fo, K));
    hipLaunchKernelGGL(k_wgrad_reduce, dim3(ceil_div(total, 256)), dim3(256), 0, st, wsf, r_ptr, S,
                       (int)Fo, (int)K, dwr, dwl, dbl);
    return launch_status();
}

extern "C" size_t ngnn_sage_dgrad_workspace_bytes(int64_t n_rows, int64_t K, int reduce) {
    if (reduce != NGNN_REDUCE_MAX || n_rows <= 0 || K <= 0) return 0;
    return sizeof(float) * static_cast<size_t>(n_rows) * static_cast<size_t>(K);
}

extern "C" int ngnn_sage_dgrad_gather(const float *dagg, int64_t ld_dagg, const float *droot,
                                      int64_t ld_droot, const int32_t *rowptr, const int32_t *col,
                                      const int32_t *rowptr_t, const int32_t *col_t, int64_t n_rows,
                                      const int32_t *r_ptr, const int32_t *rnext_ptr, int64_t K,
                                      int reduce, const float *h, int64_t ldh, const float *agg,
                                      int64_t ld_agg, float *dh, int64_t ldd, int zero_tail,
                                      void *ws, size_t ws_bytes, void *stream) {
    NGNN_RETURN_IF(reduce < NGNN_REDUCE_SUM || reduce > NGNN_REDUCE_MAX, NGNN_E_ARG);
    NGNN_RETURN_IF(!dagg || !droot || !rowptr || !rowptr_t || !r_ptr || !rnext_ptr || !dh, NGNN_E_ARG);
    NGNN_RETURN_IF(K <= 0 || n_rows < 0, NGNN_E_ARG);
    NGNN_RETURN_IF(ld_dagg < K || ld_droot < K || ldd < K, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(n_rows) || !fits_i32(K), NGNN_E_RANGE);
    if (n_rows == 0) return NGNN_OK;
    const bool is_max = reduce == NGNN_REDUCE_MAX;
    NGNN_RETURN_IF(is_max && (!h || !agg || !col), NGNN_E_ARG);
    NGNN_RETURN_IF(is_max && (ldh < K || ld_agg < K), NGNN_E_SHAPE);
    NGNN_RETURN_IF(is_max && (!ws || ws_bytes < ngnn_sage_dgrad_workspace_bytes(n_rows, K, reduce)),
                   NGNN_E_WORKSPACE);
    hipStream_t st = as_stream(stream);
    const bool vec = (K % 4 == 0) && (ld_dagg % 4 == 0) && (ld_droot % 4 == 0) && (ldd % 4 == 0) &&
                     aligned(dagg, 16) && aligned(droot, 16) && aligned(dh, 16) &&
                     (!is_max || ((ldh % 4 == 0) && (ld_agg % 4 == 0) && aligned(h, 16) &&
                                  aligned(agg, 16) && aligned(ws, 16)));
    const float *src = dagg;
    int64_t ld_src = ld_dagg;
    auto go = [&](auto vec_c, auto lpr_c) {
        constexpr int VECv = decltype(vec_c)::value;
        constexpr int LPRv = decltype(lpr_c)::value;
        const unsigned grid = static_cast<unsigned>(ceil_div(n_rows, 256 / LPRv));
        if (is_max) {
            float *gd = static_cast<float *>(ws);
            hipLaunchKernelGGL((k_max_gdist<VECv, LPRv>), dim3(grid), dim3(256), 0, st, dagg,
                               ld_dagg, rowptr, col, (int)n_rows, r_ptr, (int)K, h, ldh, agg, ld_agg,
                               gd);
            src = gd;
            ld_src = K;
            hipLaunchKernelGGL((k_dgrad_gather<VECv, LPRv, NGNN_REDUCE_MAX>), dim3(grid), dim3(256),
                               0, st, src, ld_src, droot, ld_droot, rowptr, rowptr_t, col_t,
                               (int)n_rows, r_ptr, rnext_ptr, (int)K, h, ldh, agg, ld_agg, dh, ldd,
                               zero_tail);
        } else if (reduce == NGNN_REDUCE_MEAN) {
            hipLaunchKernelGGL((k_dgrad_gather<VECv, LPRv, NGNN_REDUCE_MEAN>), dim3(grid), dim3(256),
                               0, st, src, ld_src, droot, ld_droot, rowptr, rowptr_t, col_t,
                               (int)n_rows, r_ptr, rnext_ptr, (int)K, h, ldh, agg, ld_agg, dh, ldd,
                               zero_tail);
        } else {
            hipLaunchKernelGGL((k_dgrad_gather<VECv, LPRv, NGNN_REDUCE_SUM>), dim3(grid), dim3(256),
                               0, st, src, ld_src, droot, ld_droot, rowptr, rowptr_t, col_t,
                               (int)n_rows, r_ptr, rnext_ptr, (int)K, h, ldh, agg, ld_agg, dh, ldd,
                               zero_tail);
        }
    };
    using I4 = std::integral_constant<int, 4>;
    using I1 = std::integral_constant<int, 1>;
    const int lpr = lpr_for(K, vec ? 4 : 1);
    auto dispatch_lpr = [&](auto vec_c) {
        switch (lpr) {
            case 4: go(vec_c, std::integral_constant<int, 4>{}); break;
            case 8: go(vec_c, std::integral_constant<int, 8>{}); break;
            case 16: go(vec_c, std::integral_constant<int, 16>{}); break;
            case 32: go(vec_c, std::integral_constant<int, 32>{}); break;
            default: go(vec_c, std::integral_constant<int, 64>{}); break;
        }
    };
    if (vec) dispatch_lpr(I4{});
    else dispatch_lpr(I1{});
    return launch_status();
}

extern "C" int ngnn_sage_dgrad_scatter(const float *dagg, int64_t ld_dagg, const float *droot,
                                       int64_t ld_droot, const int32_t *rowptr, const int32_t *col,
                                       int64_t n_rows, const int32_t *r_ptr,
                                       const int32_t *rnext_ptr, int64_t K, int reduce,
                                       const float *h, int64_t ldh, const float *agg,
                                       int64_t ld_agg, float *dh, int64_t ldd, int zero_tail,
                                       void *stream) {
    NGNN_RETURN_IF(reduce < NGNN_REDUCE_SUM || reduce > NGNN_REDUCE_MAX, NGNN_E_ARG);
    NGNN_RETURN_IF(!dagg || !droot || !rowptr || !r_ptr || !rnext_ptr || !dh, NGNN_E_ARG);
    NGNN_RETURN_IF(K <= 0 || n_rows < 0, NGNN_E_ARG);
    NGNN_RETURN_IF(ld_dagg < K || ld_droot < K || ldd < K, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(n_rows) || !fits_i32(K), NGNN_E_RANGE);
    if (n_rows == 0) return NGNN_OK;
    const bool is_max = reduce == NGNN_REDUCE_MAX;
    NGNN_RETURN_IF(is_max && (!h || !agg), NGNN_E_ARG);
    NGNN_RETURN_IF(is_max && (ldh < K || ld_agg < K), NGNN_E_SHAPE);
    hipStream_t st = as_stream(stream);
    dh_init_launch(droot, ld_droot, n_rows, r_ptr, rnext_ptr, K, dh, ldd, zero_tail, st);
    const unsigned g = static_cast<unsigned>(std::min<int64_t>(ceil_div(n_rows, 4), 2048));
    if (reduce == NGNN_REDUCE_MEAN)
        hipLaunchKernelGGL((k_dgrad_scatter<NGNN_REDUCE_MEAN>), dim3(g), dim3(256), 0, st, dagg,
                           ld_dagg, rowptr, col, (int)n_rows, r_ptr, (int)K, h, ldh, agg, ld_agg, dh,
                           ldd);
    else if (reduce == NGNN_REDUCE_SUM)
        hipLaunchKernelGGL((k_dgrad_scatter<NGNN_REDUCE_SUM>), dim3(g), dim3(256), 0, st, dagg,
                           ld_dagg, rowptr, col, (int)n_rows, r_ptr, (int)K, h, ldh, agg, ld_agg, dh,
                           ldd);
    else
        hipLaunchKernelGGL((k_dgrad_scatter<NGNN_REDUCE_MAX>), dim3(g), dim3(256), 0, st, dagg,
                           ld_dagg, rowptr, col, (int)n_rows, r_ptr, (int)K, h, ldh, agg, ld_agg, dh,
                           ldd);
    return launch_status();
}

static int dgrad_num_cus() {
    static int n = 0;
    if (!n) {
        int dev = 0, v = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
            v = 256;
        n = v;
    }
    return n;
}

extern "C" int ngnn_sage_dgrad_fused(const float *dy, int64_t ldy, const float *y, int64_t ldyy,
                                     float yscale, const float *wl, const float *wr, int64_t Fo,
                                     int64_t K, const int32_t *rowptr, const int32_t *col,
                                     int64_t n_rows, const int32_t *r_ptr,
                                     const int32_t *rnext_ptr, int reduce, const float *h,
                                     int64_t ldh, const float *agg, int64_t ld_agg, float *dh,
                                     int64_t ldd, int zero_tail, void *stream) {
    NGNN_RETURN_IF(reduce < NGNN_REDUCE_SUM || reduce > NGNN_REDUCE_MAX, NGNN_E_ARG);
    NGNN_RETURN_IF(!dy || !wl || !wr || !rowptr || !r_ptr || !rnext_ptr || !dh, NGNN_E_ARG);
    NGNN_RETURN_IF(Fo <= 0 || K <= 0 || n_rows < 0, NGNN_E_ARG);
    NGNN_RETURN_IF(Fo > FD_MAXF, NGNN_E_SHAPE);
    NGNN_RETURN_IF(ldy < Fo || (y && ldyy < Fo) || ldd < K, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(n_rows) || !fits_i32(K), NGNN_E_RANGE);
    if (n_rows == 0) return NGNN_OK;
    const bool is_max = reduce == NGNN_REDUCE_MAX;
    NGNN_RETURN_IF(is_max && (!h || !agg), NGNN_E_ARG);
    NGNN_RETURN_IF(is_max && (ldh < K || ld_agg < K), NGNN_E_SHAPE);
    hipStream_t st = as_stream(stream);
    dh_init_launch(nullptr, K, n_rows, r_ptr, rnext_ptr, K, dh, ldd, zero_tail, st);
    // W in LDS when both fit next to the dz slots (persistent workgroups,
    // one per CU, rows grid-strided); else the L2-streaming variant
    // -- and F_out >= 32: a narrow W (Amazon-Computers' 512 -> 10 output
    // layer: 40 KB) is as cheap from L2, and without the LDS copy the grid is
    // not held to one workgroup per CU (NGNN_DGRAD_LDSW=1 / 0, read once:
    // always / never -- A/B)
    static const int ldsw_env = [] {
        const char *e = std::getenv("NGNN_DGRAD_LDSW");
        return e ? std::atoi(e) : -1;
    }();
    const size_t wbytes = 2 * sizeof(float) * static_cast<size_t>(Fo) * static_cast<size_t>(K);
    const bool lds_w = ((Fo * K) % 4 == 0) && aligned(wl, 16) && aligned(wr, 16) &&
                       wbytes + sizeof(float) * 4 * FD_MAXF <= 150 * 1024 &&
                       (ldsw_env == 1 || (ldsw_env < 0 && Fo >= 32));
    const unsigned g = static_cast<unsigned>(
        std::min<int64_t>(ceil_div(n_rows * ceil_div(K, 64), 4), lds_w ? dgrad_num_cus() : 1024));
    auto go = [&](auto red_c, auto lds_c) {
        constexpr int RED_ = decltype(red_c)::value;
        constexpr bool L_ = decltype(lds_c)::value;
        auto fn = k_dgrad_fused<RED_, L_>;
        if (L_) {
            static bool attr = false;
            if (!attr) {
                (void)hipFuncSetAttribute(reinterpret_cast<const void *>(fn),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
                attr = true;
            }
        }
        hipLaunchKernelGGL(fn, dim3(g), dim3(256), L_ ? wbytes : 0, st, dy, ldy, y, ldyy, yscale,
                           wl, wr, (int)Fo, (int)K, rowptr, col, (int)n_rows, r_ptr, h, ldh, agg,
                           ld_agg, dh, ldd);
    };
    using RM = std::integral_constant<int, NGNN_REDUCE_MEAN>;
    using RS = std::integral_constant<int, NGNN_REDUCE_SUM>;
    using RX = std::integral_constant<int, NGNN_REDUCE_MAX>;
    using T = std::true_type;
    using Fb = std::false_type;
    if (reduce == NGNN_REDUCE_MEAN) {
        if (lds_w) go(RM{}, T{}); else go(RM{}, Fb{});
    } else if (reduce == NGNN_REDUCE_SUM) {
        if (lds_w) go(RS{}, T{}); else go(RS{}, Fb{});
    } else {
        if (lds_w) go(RX{}, T{}); else go(RX{}, Fb{});
    }
    return launch_status();
}

// the narrow scatter alone (ngnn_sage2_bwd, ngnn_bwd2.hip): g[col[e]] +=
// dy[d] (/ deg(d)) over target rows d < *r_ptr, no weight-image blocks
namespace ngnn {
int lowdim_scatter_launch(const float *dy, int64_t ldy, const int32_t *rowptr, const int32_t *col, int n_rows,
                          const int32_t *r_ptr, int Fo, int C4, float *g, int mean, hipStream_t st) {
    const int gs = static_cast<int>(std::min<int64_t>(ceil_div(n_rows, 4), 2048));
    if (gs <= 0) return NGNN_OK;
    auto go = [&](auto mean_c) {
        hipLaunchKernelGGL((k_lowdim_scatter<decltype(mean_c)::value, false>), dim3(gs), dim3(256), 0, st, dy, ldy,
                           (const float *)nullptr, Fo, 1.0f, rowptr, col, n_rows, r_ptr, Fo, C4, g, gs,
                           (const float *)nullptr, (const float *)nullptr, int64_t{0}, 0, 0, (float *)nullptr);
    };
    if (mean) go(std::true_type{});
    else go(std::false_type{});
    return launch_status();
}
}  // namespace ngnn

// ---- low-dimensional input gradient: C ABI
static int lowdim_ntw(int64_t K) {
    const int64_t half = ceil_div(ceil_div(K, 16), 2);
    int t = 1;
    while (t < half) t <<= 1;
    return t;
}
static size_t lowdim_lds_bytes(int64_t Fo, int ntw) {
    const int64_t C4 = (Fo + 3) & ~int64_t{3};
    return sizeof(float) * static_cast<size_t>(lowdim_img_floats(Fo, 2 * ntw) + LD_ROWS * (2 * C4 + 4));
}
constexpr size_t LOWDIM_LDS_MAX = 150 * 1024;

extern "C" size_t ngnn_sage_dgrad_lowdim_workspace_bytes(int64_t n_rows, int64_t Fo, int64_t K) {
    if (n_rows <= 0 || Fo <= 0 || K <= 0) return 0;
    const size_t img = sizeof(float) * static_cast<size_t>(lowdim_img_floats(Fo, 2 * lowdim_ntw(K)));
    return ((img + 255) & ~size_t{255}) +
           sizeof(float) * static_cast<size_t>(n_rows) * static_cast<size_t>((Fo + 3) & ~int64_t{3});
}

extern "C" int ngnn_sage_dgrad_lowdim(const float *dy, int64_t ldy, const float *y, int64_t ldyy,
                                      float yscale, const float *wl, const float *wr, int64_t ldw,
                                      int64_t Fo, int64_t K, const int32_t *rowptr,
                                      const int32_t *col, int64_t n_rows, const int32_t *r_ptr,
                                      const int32_t *rnext_ptr, int reduce, float *dh, int64_t ldd,
                                      int zero_tail, void *ws, size_t ws_bytes, void *stream) {
    NGNN_RETURN_IF(reduce != NGNN_REDUCE_SUM && reduce != NGNN_REDUCE_MEAN, NGNN_E_ARG);
    NGNN_RETURN_IF(!dy || !wl || !wr || !rowptr || !col || !r_ptr || !rnext_ptr || !dh, NGNN_E_ARG);
    NGNN_RETURN_IF(Fo <= 0 || K <= 0 || n_rows < 0, NGNN_E_ARG);
    NGNN_RETURN_IF(ldy < Fo || (y && ldyy < Fo) || ldd < K || ldw < K, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(n_rows) || !fits_i32(K), NGNN_E_RANGE);
    const int ntw = lowdim_ntw(K);
    NGNN_RETURN_IF(ntw > 16 || lowdim_lds_bytes(Fo, ntw) > LOWDIM_LDS_MAX, NGNN_E_SHAPE);
    if (n_rows == 0) return NGNN_OK;
    NGNN_RETURN_IF(!ws || ws_bytes < ngnn_sage_dgrad_lowdim_workspace_bytes(n_rows, Fo, K) ||
                       !aligned(ws, 16), NGNN_E_WORKSPACE);
    hipStream_t st = as_stream(stream);
    const int C4 = static_cast<int>((Fo + 3) & ~int64_t{3});
    const int ntp = 2 * ntw;
    const int64_t img_n = lowdim_img_floats(Fo, ntp);
    float *img = static_cast<float *>(ws);
    float *g = img + (((img_n * 4 + 255) & ~int64_t{255}) >> 2);
    if (zero_tail) {  // rows >= Rn of the returned gradient
        dh_init_launch(nullptr, K, n_rows, r_ptr, rnext_ptr, K, dh, ldd, 1, st);
    }
    const int gs = static_cast<int>(std::min<int64_t>(ceil_div(n_rows, 4), 2048));
    const int gp = static_cast<int>(ceil_div(img_n, 256));
    auto scatter = [&](auto mean_c, auto mask_c) {
        hipLaunchKernelGGL((k_lowdim_scatter<decltype(mean_c)::value, decltype(mask_c)::value>),
                           dim3(gs + gp), dim3(256), 0, st, dy, ldy, y, ldyy, yscale, rowptr, col,
                           (int)n_rows, r_ptr, (int)Fo, C4, g, gs, wl, wr, ldw, (int)K, ntp, img);
    };
    using T = std::true_type;
    using Fb = std::false_type;
    const bool mean = reduce == NGNN_REDUCE_MEAN;
    if (mean) { if (y) scatter(T{}, T{}); else scatter(T{}, Fb{}); }
    else { if (y) scatter(Fb{}, T{}); else scatter(Fb{}, Fb{}); }
    int rc = launch_status();
    if (rc) return rc;
    const bool vout = (K % 4 == 0) && (ldd % 4 == 0) && aligned(dh, 16);
    const size_t lds = lowdim_lds_bytes(Fo, ntw);
    const unsigned gg = static_cast<unsigned>(
        std::max<int64_t>(1, std::min<int64_t>(dgrad_num_cus(), ceil_div(n_rows, 16))));
    auto gemm = [&](auto ntw_c, auto vout_c) {
        auto fn = k_lowdim_gemm<decltype(ntw_c)::value, decltype(vout_c)::value>;
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(fn),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, LOWDIM_LDS_MAX);
            attr = true;
        }
        hipLaunchKernelGGL(fn, dim3(gg), dim3(512), lds, st, dy, ldy, y, ldyy, yscale, img,
                           (int)Fo, (int)K, (int)n_rows, r_ptr, rnext_ptr, g, C4, dh, ldd);
    };
    auto by_ntw = [&](auto vout_c) {
        switch (ntw) {
            case 1: gemm(std::integral_constant<int, 1>{}, vout_c); break;
            case 2: gemm(std::integral_constant<int, 2>{}, vout_c); break;
            case 4: gemm(std::integral_constant<int, 4>{}, vout_c); break;
            case 8: gemm(std::integral_constant<int, 8>{}, vout_c); break;
            default: gemm(std::integral_constant<int, 16>{}, vout_c); break;
        }
    };
    if (vout) by_ntw(T{}); else by_ntw(Fb{});
    return launch_status();
}
