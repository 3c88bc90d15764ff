// Row-tile fused SAGEConv layer forward for gfx950 (the default forward path
// of ngnn_sage_fwd whenever the packed W_r fits in LDS).
//
// Same contract as the 64-row kernel in ngnn_sage.hip (one SAGEConv layer of
// sage.py:33-39: out = act(b + x W_r^T + [deg>0] agg(x) W_l^T), relu, hash
// dropout), re-decomposed for the MFMA / store-issue balance that kernel's
// ablation showed (profiles/ablation_r01: its dword-store epilogue alone ran
// at 1.85 TB/s, and the MFMA loop at ~55 % of the f32 MFMA rate):
//
//   * one 512-thread workgroup per CU, persistent; W_r (and W_l when both
//     fit) is copied ONCE per workgroup into LDS in fragment order (the
//     ngnn_pack_weight layout), bias too;
//   * each wave owns 16-row tiles: tile t -> workgroup t % G, wave
//     (t / G) % 8, so consecutive tiles (NeighborLoader puts every row with
//     in-edges first) spread over all CUs and both waves of a SIMD;
//   * MFMA operands are swapped w.r.t. the 64-row kernel: A = W (16 output
//     features from LDS, one ds_read_b128 = 4 k-steps), B = x (16 graph rows
//     straight from HBM into registers, no LDS staging, no barrier), so each
//     lane ends with 4 CONSECUTIVE output features of one row -> 16-B stores;
//   * the next tile's x fragments are prefetched before the current tile's
//     MFMAs; W fragments for the next k-step are read before the current
//     k-step's MFMAs (two register sets);
//   * tiles whose rows have in-edges gather the aggregate into registers in
//     the same lane layout (per column, edge order, then / max(deg,1): the
//     fp32 sequence of ngnn_seg_agg_fwd, so the aggregate is bit-identical),
//     neighbour indices preloaded 16 per row and broadcast by ds_bpermute.
//
// Root-term arithmetic (X3, the default): fp32-accurate 3 x bf16 split MFMA.
// x and W_r are each split v = v1 + v2 + v3 (bf16, round to nearest: |v -
// v1 - v2 - v3| <= 2^-27 |v|) and x.W_r^T is accumulated in fp32 from the six
// products whose magnitude reaches 2^-18 of the leading term (v1w1, v1w2,
// v2w1, v2w2, v1w3, v3w1; each bf16 x bf16 product is exact in fp32; the
// three dropped terms are <= 2^-26 relative) on v_mfma_f32_16x16x32_bf16:
// 6 bf16 MFMAs at 16 cycles = 96 cycles per 32-deep k-chunk vs 8 fp32
// 16x16x4 MFMAs at 32 = 256.  The error is below the fp32 rounding of the
// reference's own GEMM.  A tail of K % 32 <= 12 columns
// runs on exact fp32 MFMA steps (cheaper than a padded bf16 chunk).  With
// NGNN_MATH_EXACT_F32 OR-ed into `reduce`, every product is exact-fp32
// v_mfma_f32_16x16x4_f32 (a fmaf chain).  The neighbour term (edge tiles)
// stays on exact fp32 MFMA with W_l fp32.
//
// Bytes per launch: 4*(N*K + E*K + E + N + 1 + N*F_out) (x, gathered rows,
// col, rowptr, out) + the optional saved aggregate; flops 2*N*K*F_out +
// 2*N_edge_rows*K*F_out.
#include <cstdlib>

#include "ngnn_device.h"

#ifndef NGNN_RT_WSTREAM_DEPTH
#define NGNN_RT_WSTREAM_DEPTH 2  // (A/B build flag) W_l fragment groups in flight from L2
#endif
#ifndef NGNN_RT_MAXNTW
#define NGNN_RT_MAXNTW 16  // (A/B build flag) widest output-tile slice
#endif
#ifndef NGNN_RT_STATIC
#define NGNN_RT_STATIC 0  // (A/B build flag) 1: fixed tile-per-wave schedule
#endif
// (diagnostic builds only, never shipped: 1 drops the layer's output stores /
// its root-term MFMAs / its x loads, to time the rest of the kernel)
#ifndef NGNN_RT_DBG_NOSTORE
#define NGNN_RT_DBG_NOSTORE 0
#endif
#ifndef NGNN_RT_DBG_NOMFMA
#define NGNN_RT_DBG_NOMFMA 0
#endif
#ifndef NGNN_RT_DBG_NOLOAD
#define NGNN_RT_DBG_NOLOAD 0
#endif
#ifndef NGNN_RT_FAST_BUILD
#define NGNN_RT_FAST_BUILD 0  // (development builds) 1: the fp32 MEAN kernels only
#endif

namespace ngnn {

namespace {

constexpr int RT_ROWS = 16;  // rows per wave tile (one MFMA n-tile)
constexpr int RT_KC = 8;     // k-groups of 16 per chunk (128 columns of K)
// waves per workgroup: 2 per SIMD (<= 256 VGPRs: accumulators, the current
// and the prefetched x fragments, two W fragment sets)
constexpr int RT_WAVES = 8;
constexpr int X3_TAIL_MAX = 3;  // fp32 tail steps (K % 32 <= 12); more: a padded bf16 chunk

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// v = p1 + p2 + p3 in bf16 (round to nearest even).  GUARD: an infinite v
// gives (v, 0, 0) instead of the NaN residual inf - inf (the weight images,
// split once per launch); the per-tile split of x runs unguarded -- two VALU
// per element less on the kernel's issue-bound path -- so an infinite input
// element yields NaN where fp32 arithmetic gives +-inf or NaN.  A NaN gives
// NaNs either way.
template <bool GUARD = true>
__device__ __forceinline__ void split3(v4f a, v4f b, bf16x8 &p1, bf16x8 &p2, bf16x8 &p3) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float v = j < 4 ? a[j] : b[j - 4];
        const __bf16 h = static_cast<__bf16>(v);
        const float fh = static_cast<float>(h);
        const float r = (GUARD && fh == v) ? 0.0f : v - fh;
        const __bf16 m = static_cast<__bf16>(r);
        const float r2 = r - static_cast<float>(m);
        p1[j] = h;
        p2[j] = m;
        p3[j] = static_cast<__bf16>(r2);
    }
}

struct RtArgs {
    const float *x;
    int64_t ldx;
    int K, KG;  // KG = ceil(K / 16)
    int n_rows;
    const int32_t *n_rows_dev;
    const int32_t *tile_end_dev;  // non-null: tiles only below ceil16(*tile_end_dev) (split mode)
    const int32_t *rowptr;
    const int32_t *col;
    const v4f *wl;  // packed [NT][KG][64] or NULL (no neighbour term); raw (see ldw) only
                    // when it is staged in LDS -- streamed W_l is always packed
    const v4f *wr;  // packed [NT][KG][64] or raw (see ldw)
    int64_t ldw;    // 0: packed;  > 0: raw PyG Linear weights [F_out, K], row stride ldw
    int NT, Fo;
    float *out;
    int64_t ldo;
    int vec_out;
    float *agg_out;
    int64_t ld_agg;
    // non-null: the neighbour aggregate of every row is already in agg_in
    // (ld_agg), written by the first column slice of this layer -- later
    // slices read it densely instead of gathering again
    const float *agg_in;
    Epi epi;
    const uint64_t *seed_dev;                 // XORed into the dropout seed (HIP-graph replays)
    const float *const *x_dev;                // non-null: x's address read at run time (graph slot)
    // fused x[n_id] gather: logical row r is row xrow[r] of x (the resident
    // feature table, x_rows rows); the device word xrow_dev (graph slot)
    // overrides xrow; both null: identity
    const int64_t *xrow;
    const int64_t *const *xrow_dev;
    int64_t x_rows;
    // (with xrow) col already mapped through xrow: the gather's sources are
    // table rows, no dependent index load per neighbour
    const int32_t *col_x;
    int x_bf16;  // x (and the gathered rows) are bf16: 2-B elements, ldx in elements
    int w1;      // NGNN_W_BF16: the root image holds one weight part
    // X3 root term: C 32-deep bf16 chunks (the last one zero-padded past K
    // when kpad), then T4 exact-fp32 steps of 4 columns
    int C, T4, kpad;
    const float *wr_raw;  // X3: raw W_r rows of this slice [Fo, K], stride ldw
    // narrow mode (last layer, MEAN/SUM): output tiles [0, NT1) are W_r rows
    // (out = b + x W_r^T, the root term), tiles [NT1, NT) W_l rows written to
    // z = x W_l^T [n_rows, ldz] (the neighbour term is aggregated afterwards
    // in the F_out-wide space); NT1 == NT otherwise
    int NT1;
    const float *wz_raw;
    float *z;
    int64_t ldz;
};

// -1 (all ones) when a < b, else 0: a lane mask held in a VGPR, built without
// a compare (no SGPR lane-mask pairs to keep live across the tile loop).
// Operands stay far from overflow (|a - b| < 2^31).
__device__ __forceinline__ int lt_mask(int a, int b) { return (a - b) >> 31; }

// rowptr[16 t + rl] and rowptr[16 t + rl + 1] of tile t (uniform) by scalar
// loads: one s_load_dwordx16 + one s_load_dword for a tile inside the rows,
// clamped single loads for the last one; lane rl then selects its pair.
__device__ __forceinline__ void tile_bounds(const int32_t *rowptr, int t, int n_rows, int rl,
                                            int &beg, int &end) {
    typedef const __attribute__((address_space(4))) int32_t *cp;
    const int r0 = t * 16;
    int v[17];
    if (r0 + 16 <= n_rows) {
        const cp p = (cp)(rowptr + r0);
#pragma unroll
        for (int j = 0; j < 17; ++j) v[j] = p[j];
    } else {
        const cp p = (cp)(rowptr);
#pragma unroll
        for (int j = 0; j < 17; ++j) v[j] = p[min(r0 + j, n_rows)];
    }
    int b = v[0], e = v[1];
#pragma unroll
    for (int j = 1; j < 16; ++j) {
        b = rl == j ? v[j] : b;
        e = rl == j ? v[j + 1] : e;
    }
    beg = b;
    end = e;
}

__device__ __forceinline__ v4f and_mask(v4f v, int m) {
    v4f o;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = __int_as_float(__float_as_int(v[i]) & m);
    return o;
}

// Raw buffer access (gfx9 buffer resource: 64-bit base, byte range, stride
// 0).  Loads past the range return 0 and stores past it are dropped, so rows
// beyond n_rows and padded neighbour slots need no lane predicates; the byte
// offset is one VGPR and the per-k-group step an immediate.

// byte offset past every range (load 0 / store dropped): the whole-buffer
// resource of the gather source is capped below it (host check), every other
// resource covers one 16-row tile; offsets are unsigned 32-bit
constexpr int kOOB = static_cast<int>(0xF0000000u);
constexpr int64_t kRangeMax = 0xF0000000ll - 4096;  // largest whole-buffer range

// resource over tile t's rows of a row-major [n_rows, ld] matrix (64-bit
// base per tile: no whole-buffer size limit).  It covers the 16 rows plus
// 128 columns of the next row (the X3 / fp32 row loads read whole 128-column
// groups past K), or up to column `cols` of the last row for the last tile.
__device__ __forceinline__ i32x4 tile_rsrc(const float *base, int64_t ld, int cols, int t,
                                           int n_rows) {
    const int left = n_rows - t * 16;
    const uint32_t bytes = left > 16 ? static_cast<uint32_t>((16 * ld + 128) * 4)
                                     : static_cast<uint32_t>(((left - 1) * ld + cols) * 4) * (left > 0);
    return make_rsrc(base + static_cast<int64_t>(t) * 16 * ld, bytes);
}

// x fragments of one 128-column chunk: lane (rl, q) holds
// x[r][k0 + 16 g + 4 q .. +3]; rows past n_rows read 0 (buffer range).
// Columns past K (which read the next row) are masked by mask_x at the point
// of USE, not here: masking right after the loads would make the compiler
// wait for a prefetch the moment it is issued.
// X3 layout instead: lane (rl, q) holds x[r][k0 + 32 c + 8 q + 4 h .. +3] in
// xf[2 c + h] (the B fragment of 16x16x32 bf16: 8 consecutive k per lane);
// 32-chunks past the root term's C read nothing (offset past the range).
// rowoff: byte offset of the lane's (physical) row in x, kOOB for rows past
// the block (those read 0).
// XB (X3 only): x is bf16 -- a 32-chunk's 8 values per lane are ONE 16-B
// load, already the bf16 B operand (x = x1 exactly, x2 = x3 = 0); it lands
// in xf[2 c] (xf[2 c + 1] unused).
template <bool X3, bool XB = false>
__device__ __forceinline__ void load_x(v4f (&xf)[RT_KC], i32x4 xr, uint32_t rowoff, int k0, int q) {
    if (XB) {
        const uint32_t voff = rowoff + static_cast<uint32_t>((k0 + 8 * q) * 2);
#pragma unroll
        for (int c = 0; c < RT_KC / 2; ++c) {
            xf[2 * c] = buf_load4(xr, static_cast<int>(voff + 64 * c), 0, 0);
            xf[2 * c + 1] = v4f{0.f, 0.f, 0.f, 0.f};
        }
    } else if (X3) {
        // all four chunks unconditionally: a chunk past the root term reads
        // bytes of the same / next row (or 0 past the range) and is never
        // used -- a uniform per-chunk select here becomes loop-invariant SGPR
        // lane masks that the compiler hoists and spills
        const uint32_t voff = rowoff + static_cast<uint32_t>((k0 + 8 * q) * 4);
#pragma unroll
        for (int g = 0; g < RT_KC; ++g)
            xf[g] = buf_load4(xr, static_cast<int>(voff + 4 * (32 * (g >> 1) + 4 * (g & 1))), 0, 0);
    } else {
        const uint32_t voff = rowoff + static_cast<uint32_t>((k0 + 4 * q) * 4);
#pragma unroll
        for (int g = 0; g < RT_KC; ++g) xf[g] = buf_load4(xr, static_cast<int>(voff + 64 * g), 0, 0);
    }
}

// X3 fp32 tail: lane (rl, q) holds x[r][32 C + 4 s + q] (the B operand of
// 16x16x4 f32 step s)
template <bool XB = false>
__device__ __forceinline__ void load_xt(float (&xt)[X3_TAIL_MAX], const RtArgs &a, i32x4 xr,
                                        uint32_t rowoff, int q) {
    if (XB) {  // bf16 element e: the dword holding it (rows start on 8 B), then its half
#pragma unroll
        for (int s = 0; s < X3_TAIL_MAX; ++s) {
            const int e = 32 * a.C + 4 * s + q;
            const int w = buf_load1i(xr, static_cast<int>(rowoff + static_cast<uint32_t>((e & ~1) * 2)), 0, 0);
            xt[s] = __int_as_float((e & 1) ? (w & static_cast<int>(0xffff0000u)) : (w << 16));
        }
        return;
    }
    const uint32_t voff = rowoff + static_cast<uint32_t>((32 * a.C + q) * 4);
#pragma unroll
    for (int s = 0; s < X3_TAIL_MAX; ++s)
        xt[s] = buf_load1(xr, static_cast<int>(voff + 16 * s), 0, 0);  // masked at use
}

// root term of one 128-column group in the X3 layout: per 32-chunk, split x
// into three bf16 parts and issue the six products per output tile (W parts
// from the LDS image [3][C][NTW][64] bf16x8, piece stride pst)
// W1 (NGNN_W_BF16): the image holds only W's first part (bf16-exact
// weights, parts 2 and 3 are zero): the products with w2 / w3 are exact zeros
// and are skipped -- the remaining ones in the same order, so the sums are
// bitwise those of the three-part image
template <int NTW, bool XB = false, bool W1 = false>
__device__ __forceinline__ void mfma_group_x3(v4f (&acc)[NTW], const v4f (&xf)[RT_KC],
                                              const bf16x8 *__restrict__ sw3, int pst, int cc0,
                                              int ncc, int mask_last, int kq8, int lane) {
#pragma unroll
    for (int c = 0; c < RT_KC / 2; ++c) {
        if (W1 && c < ncc) {
            bf16x8 x1, x2, x3;
            if (XB) {
                i32x4 xw = __builtin_bit_cast(i32x4, xf[2 * c]);
                if (mask_last && c == ncc - 1) {
                    int kq = kq8;
                    asm volatile("" : "+v"(kq));
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        xw[j] &= (lt_mask(2 * j, kq) & 0xffff) | (lt_mask(2 * j + 1, kq) & static_cast<int>(0xffff0000u));
                }
                x1 = __builtin_bit_cast(bf16x8, xw);
            } else {
                v4f lo = xf[2 * c], hi = xf[2 * c + 1];
                if (mask_last && c == ncc - 1) {
                    int kq = kq8;
                    asm volatile("" : "+v"(kq));
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        lo[i] = __int_as_float(__float_as_int(lo[i]) & lt_mask(i, kq));
                        hi[i] = __int_as_float(__float_as_int(hi[i]) & lt_mask(4 + i, kq));
                    }
                }
                split3<false>(lo, hi, x1, x2, x3);
            }
            const bf16x8 *w = sw3 + (cc0 + c) * NTW * 64 + lane;
            bf16x8 wb[2];
            wb[0] = w[0];
#pragma unroll
            for (int m = 0; m < NTW; ++m) {
                if (m + 1 < NTW) wb[(m + 1) & 1] = w[(m + 1) * 64];
                __builtin_amdgcn_sched_barrier(0);
                v4f t = acc[m];
                if (!XB) {
                    t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[m & 1], x3, t, 0, 0, 0);
                    t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[m & 1], x2, t, 0, 0, 0);
                }
                acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[m & 1], x1, t, 0, 0, 0);
            }
        } else if (XB && c < ncc) {
            // bf16 x: exact in one part, so only the three products with x1
            i32x4 xw = __builtin_bit_cast(i32x4, xf[2 * c]);
            if (mask_last && c == ncc - 1) {  // padded last chunk: elements past K
                int kq = kq8;
                asm volatile("" : "+v"(kq));
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    xw[j] &= (lt_mask(2 * j, kq) & 0xffff) | (lt_mask(2 * j + 1, kq) & static_cast<int>(0xffff0000u));
            }
            const bf16x8 x1 = __builtin_bit_cast(bf16x8, xw);
            const bf16x8 *w = sw3 + (cc0 + c) * NTW * 64 + lane;
            bf16x8 wb[2][3];
            wb[0][0] = w[0];
            wb[0][1] = w[pst];
            wb[0][2] = w[2 * pst];
#pragma unroll
            for (int m = 0; m < NTW; ++m) {
                if (m + 1 < NTW) {
                    const int o = (m + 1) * 64;
                    wb[(m + 1) & 1][0] = w[o];
                    wb[(m + 1) & 1][1] = w[pst + o];
                    wb[(m + 1) & 1][2] = w[2 * pst + o];
                }
                __builtin_amdgcn_sched_barrier(0);
                v4f t = acc[m];
                t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[m & 1][2], x1, t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[m & 1][1], x1, t, 0, 0, 0);
                acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[m & 1][0], x1, t, 0, 0, 0);
            }
        } else if (!XB && c < ncc) {
            v4f lo = xf[2 * c], hi = xf[2 * c + 1];
            if (mask_last && c == ncc - 1) {  // padded last chunk: columns past K read the next row
                int kq = kq8;
                asm volatile("" : "+v"(kq));  // keep the masks here (not hoisted into SGPRs)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    lo[i] = __int_as_float(__float_as_int(lo[i]) & lt_mask(i, kq));
                    hi[i] = __int_as_float(__float_as_int(hi[i]) & lt_mask(4 + i, kq));
                }
            }
            bf16x8 x1, x2, x3;
            split3<false>(lo, hi, x1, x2, x3);
            const bf16x8 *w = sw3 + (cc0 + c) * NTW * 64 + lane;
            // W parts of tile m + 1 are read from LDS while tile m's six
            // MFMAs run (double-buffered): the reads' latency stays off the
            // matrix pipe (read just in time, each tile waited on lgkmcnt(0))
            bf16x8 wb[2][3];
            wb[0][0] = w[0];
            wb[0][1] = w[pst];
            wb[0][2] = w[2 * pst];
#pragma unroll
            for (int m = 0; m < NTW; ++m) {
                if (m + 1 < NTW) {
                    const int o = (m + 1) * 64;
                    wb[(m + 1) & 1][0] = w[o];
                    wb[(m + 1) & 1][1] = w[pst + o];
                    wb[(m + 1) & 1][2] = w[2 * pst + o];
                }
                // (keeps the scheduler from sinking those reads down to their use)
                __builtin_amdgcn_sched_barrier(0);
                const bf16x8 w1 = wb[m & 1][0], w2 = wb[m & 1][1], w3 = wb[m & 1][2];
                v4f t = acc[m];
                t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w3, x1, t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, x3, t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2, x2, t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2, x1, t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, x2, t, 0, 0, 0);
                acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, x1, t, 0, 0, 0);
            }
        }
    }
}

__device__ __forceinline__ void mask_x(v4f (&xc)[RT_KC], const v4f (&xf)[RT_KC], const RtArgs &a,
                                       int k0, int q) {
    const int kq = a.K - k0 - 4 * q;  // columns left for this lane's 4-wide slot
#pragma unroll
    for (int g = 0; g < RT_KC; ++g) xc[g] = and_mask(xf[g], lt_mask(16 * g, kq));
}

// Raw (PyG [F_out, K]) weights: fragment (m, kg) lane l is the 16-B run
// W[m*16 + (l & 15)][kg*16 + 4 (l >> 4) .. +3]; lanes outside F_out x K read
// row 0 / column 0 and are zeroed.  Returns the float offset; *ok the mask.
__device__ __forceinline__ int64_t raw_frag_off(int m, int kg, int lane, int64_t ldw, int Fo, int K,
                                                bool *ok) {
    const int n = m * 16 + (lane & 15), k = kg * 16 + 4 * (lane >> 4);
    *ok = n < Fo && k < K;
    return *ok ? static_cast<int64_t>(n) * ldw + k : 0;
}

// W fragment loads for k-group kg, m-tiles [p*H, p*H + H).
// LDS image: k-group major, [KG][NTW][64] v4f, so for a fixed chunk every
// (g, m) offset is a compile-time immediate off one per-chunk base (no
// per-fragment address registers); reads past the image (k-groups beyond a
// short last chunk, whose MFMAs are skipped) return LDS garbage or 0, never
// fault.  Global (W_l that does not fit): the packed [NT][KG][64] layout,
// k-group clamped and padded tiles re-read a valid one (never stored).
template <int NTW, int H, bool LDSW>
__device__ __forceinline__ void load_w(v4f (&w)[H], const v4f *__restrict__ wsrc, int KG, int kg,
                                       int p, int NT, int lane) {
#pragma unroll
    for (int h = 0; h < H; ++h) {
        const int m = p * H + h;
        if (LDSW) {
            w[h] = wsrc[(kg * NTW + m) * 64 + lane];
        } else {  // streamed from L2: always the packed layout (1 KiB per wave-load)
            w[h] = wsrc[(static_cast<int64_t>(min(m, NT - 1)) * KG + min(kg, KG - 1)) * 64 + lane];
        }
    }
}

template <int NTW, bool LDSW>
__device__ __forceinline__ void mfma_chunk_rt(v4f (&acc)[NTW], const v4f (&xf)[RT_KC],
                                              const v4f *__restrict__ wsrc, int KG, int kg0,
                                              int nkg, int NT, int lane) {
    if (!LDSW) {  // streamed: address clamps per call, not hoisted as SGPR masks
        asm volatile("" : "+s"(NT));
        asm volatile("" : "+s"(KG));
    }
    // fragments per load group (double-buffered): 4 from LDS, 2 streamed
    // from L2 (the streamed path's address registers are the tighter budget)
    constexpr int P = NTW >= 8 ? NTW / (LDSW ? 4 : 2) : 1;
    constexpr int H = NTW / P;
    // NB-deep ring: groups s + 1 .. s + NB - 1 in flight while group s's
    // MFMAs run (L2 latency is ~10x a group's MFMA time when streamed)
    constexpr int NB = LDSW ? 2 : NGNN_RT_WSTREAM_DEPTH;
    constexpr int NS = RT_KC * P;
    v4f wb[NB][H];
#pragma unroll
    for (int s = 0; s < NB - 1; ++s)
        if (s < NS) load_w<NTW, H, LDSW>(wb[s], wsrc, KG, kg0 + s / P, s % P, NT, lane);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int g = s / P, p = s % P;
        const int sn = s + NB - 1, gn = sn / P, pn = sn % P;
        if (sn < NS) load_w<NTW, H, LDSW>(wb[sn % NB], wsrc, KG, kg0 + gn, pn, NT, lane);
        if (LDSW) __builtin_amdgcn_sched_barrier(0);  // keep the next group's reads ahead
        if (g < nkg) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int h = 0; h < H; ++h)
                    acc[p * H + h] = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[s % NB][h][i], xf[g][i],
                                                                          acc[p * H + h], 0, 0, 0);
        }
    }
}

// max of v over the 16 lanes of row-group 0 (every row-group holds the same
// 16 row values here): 4 DPP row shifts, no LDS round trips
__device__ __forceinline__ int rowgroup_max16(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true));  // row_shr:1
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true));  // row_shr:2
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true));  // row_shr:4
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true));  // row_shr:8
    return __builtin_amdgcn_readlane(v, 15);
}

template <int RED>
__device__ __forceinline__ float red_op(float acc, float v) {
    return (RED == NGNN_REDUCE_MAX) ? nanmax(acc, v) : acc + v;
}

// aggregate of rows r over columns [k0, k0 + 16 nkg) into ag (same lane
// layout as load_x).  cb: this lane's 4 preloaded neighbour indices
// (lane (rl, q) holds neighbours 4q..4q+3 of its row within the current
// 16-neighbour window).
template <int RED>
__device__ __forceinline__ v4f red_mask(v4f v, int m) {
    // masked slots contribute the reduction's identity: +0.0 for sum (the
    // running sum starts at +0.0, so it is never -0.0 and s + 0.0 == s
    // bitwise), -inf for max (nanmax(s, -inf) == s)
    if (RED == NGNN_REDUCE_MAX) {
        v4f o;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            o[i] = __int_as_float((__float_as_int(v[i]) & m) | (~m & static_cast<int>(0xff800000u)));
        return o;
    }
    return and_mask(v, m);
}

// aggregate of row r over columns [k0, k0 + 128) into ag (same lane layout
// as load_x).  Neighbour indices are preloaded 16 per row (lane (rl, q)
// holds neighbours e0 + 4q .. +3 of its row) and broadcast by ds_bpermute;
// two neighbours' fragments are in flight at a time.  Per column the
// reduction runs in edge order from the identity, then / max(deg, 1) for
// mean: the fp32 sequence of ngnn_seg_agg_fwd.  Padded slots point past the
// buffer range (read 0 = the sum identity; max masks them to -inf).
// Columns past K accumulate garbage from the next row and are zeroed at the
// end.
template <int RED, bool XB = false>
__device__ __forceinline__ void gather_chunk(v4f (&ag)[RT_KC], const RtArgs &a, i32x4 xr, int beg,
                                             int deg, int maxdeg, int k0, int nkg, int rl, int q,
                                             const int64_t *xrow) {
    constexpr uint32_t EB = XB ? 2u : 4u;  // bytes per x element
    const float ident = (RED == NGNN_REDUCE_MAX) ? -INFINITY : 0.0f;
#pragma unroll
    for (int g = 0; g < RT_KC; ++g) ag[g] = v4f{ident, ident, ident, ident};
    const uint32_t kofs = static_cast<uint32_t>(k0 + 4 * q) * EB;
    const uint32_t ld4 = static_cast<uint32_t>(a.ldx) * EB;  // (whole-buffer offsets < 3.75 GiB)
#pragma unroll 1
    for (int e0 = 0; e0 < maxdeg; e0 += 16) {
        int cb[4];
        const int32_t *cl = a.col_x ? a.col_x : a.col;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = e0 + 4 * q + j;
            cb[j] = cl[(beg + e) & lt_mask(e, deg)];  // invalid slots read col[0]
        }
        if (xrow && !a.col_x) {  // fused x[n_id]: the neighbours' rows in the feature table
#pragma unroll
            for (int j = 0; j < 4; ++j) cb[j] = static_cast<int>(gload(xrow, cb[j]));
        }
        const int ne = min(16, maxdeg - e0);
#pragma unroll 1  // one neighbour pair in flight: keep the register budget
        for (int e4 = 0; 4 * e4 < ne; ++e4) {
            const int srcl = rl + 16 * e4;
#pragma unroll
            for (int j = 0; j < 4; j += 2) {
                const int e = e0 + 4 * e4 + j;
                const int m0 = lt_mask(e, deg), m1 = lt_mask(e + 1, deg);
                const int o0 = m0 ? static_cast<int>(static_cast<uint32_t>(__shfl(cb[j], srcl)) * ld4 + kofs)
                                  : kOOB;
                const int o1 = m1 ? static_cast<int>(static_cast<uint32_t>(__shfl(cb[j + 1], srcl)) * ld4 + kofs)
                                  : kOOB;
                // all 8 k-groups unconditionally (conditional writes into the
                // fragment arrays make the compiler copy them whole); groups
                // past K read the next row or 0 and are zeroed at the end
                v4f v0[RT_KC], v1[RT_KC];
#pragma unroll
                for (int g = 0; g < RT_KC; ++g) {
                    if (XB) {  // 4 bf16 per lane and k-group: one 8-B load, widened exactly
                        v0[g] = bf16x4_to_f32(buf_load2i(xr, o0 + 32 * g, 0, 0));
                        v1[g] = bf16x4_to_f32(buf_load2i(xr, o1 + 32 * g, 0, 0));
                    } else {
                        v0[g] = buf_load4(xr, o0 + 64 * g, 0, 0);
                        v1[g] = buf_load4(xr, o1 + 64 * g, 0, 0);
                    }
                }
#pragma unroll
                for (int g = 0; g < RT_KC; ++g) {
                    {
                        v4f w0 = v0[g], w1 = v1[g];
                        if (RED == NGNN_REDUCE_MAX) {
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                w0[i] = __int_as_float((__float_as_int(w0[i]) & m0) |
                                                       (~m0 & static_cast<int>(0xff800000u)));
                                w1[i] = __int_as_float((__float_as_int(w1[i]) & m1) |
                                                       (~m1 & static_cast<int>(0xff800000u)));
                            }
                        }
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            ag[g][i] = red_op<RED>(ag[g][i], w0[i]);
                            ag[g][i] = red_op<RED>(ag[g][i], w1[i]);
                        }
                    }
                }
            }
        }
    }
    // finalize: mean divides once (as scatter mean); max of nothing -> 0;
    // columns past K exactly 0 (the W padding is 0 too)
    const float dv = static_cast<float>(deg > 1 ? deg : 1);
    const int mdeg = lt_mask(0, deg);
    const int kq = a.K - k0 - 4 * q;
#pragma unroll
    for (int g = 0; g < RT_KC; ++g) {
        v4f v = ag[g];
        if (RED == NGNN_REDUCE_MEAN) {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = v[i] / dv;
        }
        ag[g] = and_mask(v, (RED == NGNN_REDUCE_MAX ? mdeg : -1) & lt_mask(16 * g, kq));
    }
}

// keep mask of bit `b` of a hash word: 0 or all ones (v_bfe_i32 through asm:
// written as shifts the compiler turns the AND with it into a compare +
// select per element)
template <int B>
__device__ __forceinline__ int bit_mask(uint32_t w) {
    int k;
    asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(k) : "v"(w), "n"(B));
    return k;
}
// (b a constant after unrolling: the switch folds to one case)
__device__ __forceinline__ int bit_mask_at(uint32_t w, int b) {
    switch (b) {
        case 0: return bit_mask<0>(w);
        case 1: return bit_mask<1>(w);
        case 2: return bit_mask<2>(w);
        default: return bit_mask<3>(w);
    }
}

// epilogue: lane holds output features m*16 + 4q .. +3 of row r.  Stores go
// through a buffer resource (rows past n_rows are dropped by the range);
// `vec` (uniform): F_out a multiple of 16 with 16-B aligned rows -- one
// 16-B store per m-tile, no per-lane predicates.  Branch-free.
// DM (dropout mode, ngnn_device.h): 0 none; 1 byte mode -- the lane's four
// columns f .. f+3 (f = col_base + 16 m + 4 q, col_base a multiple of 16) are
// one hash quad, pb + 4 m; 2 bit mode (p = 0.5) -- column c is bit c & 31 of
// hash word c >> 5, so two consecutive 16-column tiles share one word and the
// lane's four bits of tile m sit at 16 (gc & 1) + 4 q (gc = the global
// 16-column tile): one shift per tile, then four immediate bit fields.  In
// bit mode sbias holds 2 b: the survivor scale 2 is folded into the bias
// add, fma(acc, 2, 2 b) == 2 (acc + b) bitwise, and ReLU is an INTEGER max
// with 0 (a pre-activation with the sign bit set -- negative, -0.0 or a
// negative-signed NaN -- gives +0.0; a positive NaN passes), then one AND
// with the keep mask: ~4 VALU per element instead of ~9.
template <int NTW, int DM, bool RELU, bool VEC>
__device__ __forceinline__ void epilogue(const v4f (&acc)[NTW], const RtArgs &a, i32x4 orsrc,
                                         i32x4 zr, const float *sbias, int r, int rl, int q) {
    // orsrc / zr: the tile's output / z rows (rl = row in the tile); r, the
    // global row, keys the dropout hash
    const uint32_t thresh = a.epi.drop.thresh;
    const float scale = a.epi.drop.scale;
    const uint32_t rk = DM ? a.epi.drop.row_key(static_cast<uint32_t>(r)) : 0u;
    const uint32_t pb = DM == 1 ? rk + static_cast<uint32_t>((a.epi.col_base + 4 * q) >> 2) : 0u;
    const int cb16 = a.epi.col_base >> 4;  // global 16-column tile of m = 0 (uniform)
    uint32_t hw = 0;                       // bit mode: the current hash word
    const int obase = rl * static_cast<int>(a.ldo) * 4;
    // re-materialised per call: the per-tile-index tests below must not be
    // hoisted out of the tile loop as SGPR lane masks (they spill)
    int NT = a.NT, NT1 = a.NT1;
    asm volatile("" : "+s"(NT));
    asm volatile("" : "+s"(NT1));
#pragma unroll
    for (int m = 0; m < NTW; ++m) {
        if (m >= NT) continue;  // padded tiles (uniform)
        if (m >= NT1) {         // narrow mode: z = x W_l^T rows, no epilogue
            buf_store4(acc[m], zr, (rl * static_cast<int>(a.ldz) + (m - NT1) * 16 + 4 * q) * 4, 0, 0);
            continue;
        }
        const int f = m * 16 + 4 * q;
        const v4f b = *reinterpret_cast<const v4f *>(sbias + f);
        const int gc = cb16 + m;  // global 16-column tile (uniform)
        uint32_t hs = 0;          // bit mode: this lane's four bits of tile m in bits 0..3
        if (DM == 2) {
            if (m == 0 || (gc & 1) == 0) hw = lowbias32(rk + static_cast<uint32_t>(gc >> 1));
            hs = hw >> (((gc & 1) << 4) + 4 * q);
        }
        const uint32_t h = DM == 1 ? lowbias32(pb + 4u * m) : 0u;
        v4f v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (DM == 2) {
                int yi = __float_as_int(__builtin_fmaf(acc[m][j], 2.0f, b[j]));
                if (RELU) yi = max(yi, 0);
                v[j] = __int_as_float(yi & bit_mask_at(hs, j));
            } else {
                const float y = acc[m][j] + b[j];
                // y < 0 (ReLU; NaN passes, like torch.relu) or a dropped column -> 0
                bool zero = RELU && y < 0.0f;
                if (DM == 1) zero = zero || ((h >> (8 * j)) & 0xffu) < thresh;
                v[j] = zero ? 0.0f : (DM == 1 ? y * scale : y);
            }
        }
        if (NGNN_RT_DBG_NOSTORE && v[0] != 1234.5f) continue;
        if (VEC) {
            buf_store4(v, orsrc, obase + 4 * f, 0, 0);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                buf_store1(v[j], orsrc, f + j < a.Fo ? obase + 4 * (f + j) : kOOB, 0, 0);
        }
    }
}

// WLM: W_l source -- 0 streamed from L2 (packed fragments), 1 in LDS.  (A
// raw-layout L2 stream that saves the pack launch measured slower: 0.373 vs
// 0.355 ms/step on products, the extra address VALU spills the L0 kernel.)
// X3: root term on the 3 x bf16 split (LDS image of W_r split in the
// prologue from the raw rows); otherwise exact fp32 MFMA.
template <int NTW, int RED, int WLM, bool X3, bool VEC, bool XB, bool W1>
__global__ __launch_bounds__(RT_WAVES * 64) void k_sage_rt(RtArgs a) {
    static_assert(!XB || X3, "bf16 rows feed the split-bf16 root term");
    static_assert(!W1 || X3, "one weight part: the split-bf16 image");
    constexpr int NP = W1 ? 1 : 3;  // weight parts in the image
    constexpr uint32_t EB = XB ? 2u : 4u;  // bytes per x element
    constexpr bool WL_LDS = WLM == 1;
    extern __shared__ __attribute__((aligned(16))) v4f lds[];
    __shared__ int s_next_tile;       // the workgroup's tile-claim counter
    if (threadIdx.x == 0) s_next_tile = RT_WAVES;  // each wave's first tile is fixed
    const int nfr = NTW * a.KG * 64;  // fragments per fp32 weight matrix (NTW tiles, zero padded)
    // X3 image: [NP][C][NTW][64] bf16x8 (16 B each) + fp32 tail [T4][NTW][64]
    const int pst = a.C * NTW * 64;                        // bf16x8 per piece
    const int x3_v4f = X3 ? NP * pst + (a.T4 * NTW * 64) / 4 : 0;
    bf16x8 *sw3 = reinterpret_cast<bf16x8 *>(lds);
    float *swt = reinterpret_cast<float *>(lds + NP * pst);
    v4f *swr = lds;                                        // fp32 W_r image (X3 == false)
    v4f *swl = lds + (X3 ? x3_v4f : nfr);
    float *sbias = reinterpret_cast<float *>(swl + (WL_LDS ? nfr : 0));
    const int have_l = a.wl != nullptr;
    // (wave index uniform: readfirstlane, so tile indices and the per-tile
    // buffer resources derived from them stay scalar -- no waterfall loops)
    const int wv = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int ln = threadIdx.x & 63;
    {
        const int nch = a.NT * a.KG;  // valid 1-KiB fp32 fragments per matrix
        if (X3) {
            // W_r split into three bf16 parts, one lane fragment (8 consecutive
            // k of one output row) per slot; rows past F_out / columns past K
            // are zero
            // image row n: W_r row n (tiles < NT1), W_l row n - 16 NT1 (narrow
            // mode's tiles [NT1, NT)), nothing for padded tiles (>= NT) or
            // rows past F_out of either half
            auto wrow = [&](int n) -> const float * {
                if (n >= 16 * a.NT) return nullptr;
                const bool zt = n >= 16 * a.NT1;
                const int nn = zt ? n - 16 * a.NT1 : n;
                const float *base = zt ? a.wz_raw : a.wr_raw;
                if (nn >= a.Fo || base == nullptr) return nullptr;
                return base + static_cast<int64_t>(nn) * a.ldw;
            };
            const int nslot = pst;
            for (int sl = threadIdx.x; sl < nslot; sl += RT_WAVES * 64) {
                const int l = sl & 63, mt = (sl >> 6) % NTW, cc = (sl >> 6) / NTW;
                const int n = mt * 16 + (l & 15), k = 32 * cc + 8 * (l >> 4);
                v4f lo{0.f, 0.f, 0.f, 0.f}, hi{0.f, 0.f, 0.f, 0.f};
                const float *row = wrow(n);
                if (row) {
                    const float *src = row + k;
                    if (k + 8 <= a.K) {
                        lo = *reinterpret_cast<const v4f *>(src);
                        hi = *reinterpret_cast<const v4f *>(src + 4);
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            lo[j] = k + j < a.K ? src[j] : 0.0f;
                            hi[j] = k + 4 + j < a.K ? src[4 + j] : 0.0f;
                        }
                    }
                }
                bf16x8 p1, p2, p3;
                split3(lo, hi, p1, p2, p3);
                sw3[sl] = p1;
                if (!W1) {
                    sw3[pst + sl] = p2;
                    sw3[2 * pst + sl] = p3;
                }
            }
            const int ntail = a.T4 * NTW * 64;
            for (int sl = threadIdx.x; sl < ntail; sl += RT_WAVES * 64) {
                const int l = sl & 63, mt = (sl >> 6) % NTW, st = (sl >> 6) / NTW;
                const int n = mt * 16 + (l & 15), k = 32 * a.C + 4 * st + (l >> 4);
                const float *row = wrow(n);
                swt[sl] = (row && k < a.K) ? row[k] : 0.0f;
            }
        }
        // fp32 images by LDS-DMA, 1 KiB (one n-tile x k-group fragment) per
        // wave-instruction, all in flight at once; padding tiles zeroed.
        // X3: only W_l (when it lives in LDS); otherwise W_r and W_l.
        for (int c = wv; c < nch; c += RT_WAVES) {
            const int m = c / a.KG, kg = c - m * a.KG;  // [NT][KG] -> LDS [KG][NTW]
            const int d = (kg * NTW + m) * 64;
            bool ok = true;
            const int64_t so = a.ldw ? raw_frag_off(m, kg, ln, a.ldw, a.Fo, a.K, &ok) / 4
                                     : static_cast<int64_t>(c) * 64 + ln;  // in v4f units
            // (raw rows are 16-B aligned: K % 4 == 0 and ldw % 4 == 0)
            if (!X3)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(a.wr + so),
                    (__attribute__((address_space(3))) void *)(swr + d), 16, 0, 0);
            if (WL_LDS && have_l)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(a.wl + so),
                    (__attribute__((address_space(3))) void *)(swl + d), 16, 0, 0);
        }
        if (a.ldw && (!X3 || (WL_LDS && have_l))) {
            // raw weights: lanes outside F_out x K loaded row 0 / column 0 --
            // zero those slots once this wave's LDS-DMAs have landed
            __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0)
            const v4f z0{0.f, 0.f, 0.f, 0.f};
            for (int c = wv; c < nch; c += RT_WAVES) {
                const int m = c / a.KG, kg = c - m * a.KG;
                const int d = (kg * NTW + m) * 64;
                bool ok;
                (void)raw_frag_off(m, kg, ln, a.ldw, a.Fo, a.K, &ok);
                if (!ok) {
                    if (!X3) swr[d + ln] = z0;
                    if (WL_LDS && have_l) swl[d + ln] = z0;
                }
            }
        }
        const v4f z{0.f, 0.f, 0.f, 0.f};
        const int npad = (NTW - a.NT) * 64;  // padded tiles of every k-group
        for (int i = threadIdx.x; i < a.KG * npad; i += RT_WAVES * 64) {
            const int kg = i / npad, j = i - kg * npad;
            if (!X3) swr[kg * NTW * 64 + a.NT * 64 + j] = z;
            if (WL_LDS) swl[kg * NTW * 64 + a.NT * 64 + j] = z;
        }
        if (WL_LDS && !have_l)
            for (int i = threadIdx.x; i < nfr; i += RT_WAVES * 64) swl[i] = z;
        // (bit-mode dropout folds its survivor scale 2 into the bias add: 2 b)
        const float bsc = a.epi.drop.thresh == 128u ? 2.0f : 1.0f;
        for (int i = threadIdx.x; i < NTW * 16; i += RT_WAVES * 64)
            sbias[i] = (a.epi.bias && i < a.Fo) ? a.epi.bias[i] * bsc : 0.0f;
    }
    __syncthreads();

    const int wave = wv;
    int n_rows = a.n_rows;
    if (a.n_rows_dev) n_rows = min(n_rows, *a.n_rows_dev);
    const int n_tiles = (n_rows + RT_ROWS - 1) / RT_ROWS;
    // 128-column groups of the root term: X3 covers 32 C columns (at least
    // one group, which also carries the next tile's prefetch); fp32 all of K
    const int nchunk = X3 ? max(1, (a.C + 3) / 4) : (a.KG + RT_KC - 1) / RT_KC;
    const int nchunk_l = (a.KG + RT_KC - 1) / RT_KC;  // neighbour term (fp32 layout)
    const int tstride = gridDim.x * RT_WAVES;

    // tile k of this wave: k = 0 -> w0; later rounds in reverse wave order,
    // so the partial last round lands on the waves that did NOT start with a
    // (heavier) edge tile -- NeighborLoader puts the rows with in-edges
    // first (measured: -0.3..0.4 % step time)
    const int w0 = blockIdx.x + gridDim.x * wave;
    auto tile_of = [&](int k) { return k == 0 ? w0 : k * tstride + (tstride - 1 - w0); };
    // dynamic scheduling inside the workgroup: the workgroup owns tiles
    // blockIdx.x + j gridDim.x (round-robin over workgroups, as before) and
    // its waves claim them one at a time from an LDS counter -- the rows with
    // in-edges come first in a NeighborLoader block and their tiles take
    // several times longer, so a fixed tile-per-wave map leaves the waves
    // that drew them finishing last.  (A chip-wide counter in global memory
    // serialises ~10k same-address atomics: measured 2x slower.)  A wave
    // claims its next tile when it starts the current one.
    auto claim = [&]() -> int {
        int j = 0;
        if ((threadIdx.x & 63) == 0) j = atomicAdd(&s_next_tile, 1);
        return static_cast<int>(blockIdx.x) +
               __builtin_amdgcn_readfirstlane(__shfl(j, 0)) * static_cast<int>(gridDim.x);
    };
    (void)tile_of;
    int kt = 0;
#if NGNN_RT_STATIC
    int t = tile_of(0);
#else
    int t = static_cast<int>(blockIdx.x) + wave * static_cast<int>(gridDim.x);  // first claims: waves 0..7
#endif
    int tnext = 0;
    // next tile's chunk-0 x fragments and row bounds, loaded one tile ahead,
    // unconditionally (a tile past the end re-reads tile 0: valid, unused)
    v4f xn[RT_KC];
#pragma unroll
    for (int g = 0; g < RT_KC; ++g) xn[g] = v4f{0.f, 0.f, 0.f, 0.f};
    float xtn[X3_TAIL_MAX] = {0.f, 0.f, 0.f};
    int nbeg = 0, nend = 0, nmask = 0;
    if (a.seed_dev) a.epi.drop.reseed(*a.seed_dev);
    // x: the address given at launch, or (graph replay of a changing batch)
    // the one the slot load stored, ranged by the device row count
    const void *xbase = a.x_dev ? *a.x_dev : a.x;
    const int64_t *xrow = a.xrow_dev ? *a.xrow_dev : a.xrow;
    // one resource over all of x (root rows and gathered neighbour rows;
    // x_rows: the feature table's rows under the fused x[n_id] gather)
    const int64_t xrows = xrow ? a.x_rows : static_cast<int64_t>(n_rows);
    const i32x4 xr = make_rsrc(xbase, static_cast<uint32_t>(((xrows - 1) * a.ldx + a.K) * EB * (xrows > 0)));
    const uint32_t ld4 = static_cast<uint32_t>(a.ldx) * EB;
    // byte offset of logical row rr in x (kOOB past the block's rows)
    // The two forms stay separate branches (the empty asm pins each result
    // inside its branch): with one multiply after the join, the wait for
    // the n_id load sat at the join and every tile paid a vmcnt(0) -- a drain
    // of the previous tile's output stores -- even without the fused gather.
    auto row_off = [&](int rr) -> uint32_t {
        if (rr >= n_rows) return static_cast<uint32_t>(kOOB);
        uint32_t o;
        if (xrow) {
            o = static_cast<uint32_t>(gload(xrow, rr)) * ld4;
            asm volatile("; row_off n_id" : "+v"(o));
        } else {
            o = static_cast<uint32_t>(rr) * ld4;
            asm volatile("; row_off rows" : "+v"(o));
        }
        return o;
    };
    uint32_t roff_n = 0;   // the next tile's row offset (its rows are in flight)
    uint32_t roff_nn = 0;  // the claimed tile's row offset, computed when claimed: under the
                           // fused gather its xrow[] load then lands behind the current tile
    // per-lane indices are re-derived per tile from threadIdx (behind an
    // empty asm, so nothing derived from them is hoisted and kept live across
    // the tile loop: such invariants were the VGPR spills, and their reloads
    // drained the prefetch with a vmcnt(0))
    auto lane_ids = [&](int &lane_, int &q_, int &rl_) {
        int l = static_cast<int>(threadIdx.x) & 63;
        asm volatile("" : "+v"(l));
        lane_ = l;
        q_ = l >> 4;
        rl_ = l & 15;
    };
    auto prefetch = [&](int tn, uint32_t roff_tn) {
        int lane, q, rl;
        lane_ids(lane, q, rl);
        (void)lane;
        const int tl = tn < n_tiles ? tn : 0;
        const int rn = tl * RT_ROWS + rl;
        roff_n = roff_tn;
        if (NGNN_RT_DBG_NOLOAD) {
#pragma unroll
            for (int g = 0; g < RT_KC; ++g) xn[g] = v4f{float(tn), float(g), float(rl), 1.f};
        } else {
            load_x<X3, XB>(xn, xr, roff_n, 0, q);
            if (X3) load_xt<XB>(xtn, a, xr, roff_n, q);
        }
        if (have_l) {
            // the tile's 17 row bounds by SCALAR loads (the tile index is
            // uniform): they count on lgkmcnt, so using them never waits for
            // vector memory -- a per-lane vector load here made the next use
            // wait vmcnt(0), draining the x fragments just issued and the
            // previous tile's output stores
            nmask = lt_mask(rn, n_rows);  // rows past the end: degree 0 (at use)
            tile_bounds(a.rowptr, tl, n_rows, rl, nbeg, nend);
        }
    };
    {
        int lane0, q0, rl0;
        lane_ids(lane0, q0, rl0);
        prefetch(t, row_off(t * RT_ROWS + rl0));
        // Settle the first tile's loads HERE, once per wave.  The compiler's
        // wait for a loop-carried load takes the fewest younger memory ops
        // over the paths into the loop: left pending on this entry path (no
        // stores behind it), every tile's first use of its prefetched x
        // waited for the previous tile's output stores too -- a full store
        // drain per tile.
#pragma unroll
        for (int g = 0; g < RT_KC; ++g) asm volatile("" : "+v"(xn[g]));
#pragma unroll
        for (int s2 = 0; s2 < X3_TAIL_MAX; ++s2) asm volatile("" : "+v"(xtn[s2]));
        asm volatile("" : "+v"(nbeg), "+v"(nend));
    }
    for (; t < n_tiles; t = tnext, ++kt) {
#if NGNN_RT_STATIC
        tnext = tile_of(kt + 1);
        (void)claim;
#else
        tnext = claim();
#endif
        const uint32_t roff = roff_n;  // this tile's row offset (prefetch overwrites roff_n)
        int lane, q, rl;
        lane_ids(lane, q, rl);
        roff_nn = row_off(tnext * RT_ROWS + rl);
        // X3: columns of the padded last chunk this lane may keep (8 q .. 8 q + 7)
        const int kq8 = a.K - (32 * (a.C - 1) + 8 * q);
        const int r = t * RT_ROWS + rl;
        const int beg = nbeg, deg = (nend - nbeg) & nmask;
        const int maxdeg = have_l ? rowgroup_max16(deg) : 0;
        v4f acc[NTW];
#pragma unroll
        for (int m = 0; m < NTW; ++m) acc[m] = v4f{0.f, 0.f, 0.f, 0.f};
        if (X3) {
            // fp32 tail steps (the K % 32 columns past the bf16 chunks) first,
            // while the prefetched tail values are still this tile's
#pragma unroll
            for (int s2 = 0; s2 < X3_TAIL_MAX; ++s2) {
                if (s2 < a.T4) {
                    const float xv = __int_as_float(__float_as_int(xtn[s2]) &
                                                    lt_mask(32 * a.C + 4 * s2 + q, a.K));
#pragma unroll
                    for (int m = 0; m < NTW; ++m)
                        acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(swt[(s2 * NTW + m) * 64 + lane], xv,
                                                                      acc[m], 0, 0, 0);
                }
            }
        }

        // ---- root term: x[r] . W_r^T, chunk by chunk; chunk c+1 (or, in the
        // last chunk, the next tile's chunk 0 and row bounds) loads behind
        // chunk c's MFMAs
        for (int c = 0; c < nchunk; ++c) {
            v4f xc[RT_KC];
            if (X3) {
#pragma unroll
                for (int g = 0; g < RT_KC; ++g) xc[g] = xn[g];
            } else {
                mask_x(xc, xn, a, c * RT_KC * 16, q);
            }
            const int nkg = min(RT_KC, a.KG - c * RT_KC);
            if (c + 1 < nchunk) {
                load_x<X3, XB>(xn, xr, roff, (c + 1) * RT_KC * 16, q);
            } else if (maxdeg == 0) {
                prefetch(tnext, roff_nn);  // next tile: a whole tile of MFMAs to land
            }
            if (NGNN_RT_DBG_NOMFMA) {
#pragma unroll
                for (int m = 0; m < NTW; ++m) acc[m] += xc[m % RT_KC];
            } else if (X3) {
                const int ncc = min(4, a.C - 4 * c);
                mfma_group_x3<NTW, XB, W1>(acc, xc, sw3, pst, 4 * c, ncc, a.kpad && c == nchunk - 1, kq8, lane);
            } else {
                mfma_chunk_rt<NTW, true>(acc, xc, swr, a.KG, c * RT_KC, nkg, a.NT, lane);
            }
        }

        // ---- neighbour term (tiles with in-edges only)
        if (maxdeg > 0) {
            const i32x4 ar = tile_rsrc(a.agg_out, a.ld_agg, a.K, t, n_rows);
            for (int c = 0; c < nchunk_l; ++c) {
                const int k0 = c * RT_KC * 16;
                const int nkg = min(RT_KC, a.KG - c * RT_KC);
                v4f ag[RT_KC];
                if (a.agg_in) {
                    const i32x4 air = tile_rsrc(a.agg_in, a.ld_agg, a.K, t, n_rows);
                    v4f av[RT_KC];
                    load_x<false>(av, air, static_cast<uint32_t>(rl * a.ld_agg * 4), k0, q);
                    mask_x(ag, av, a, k0, q);
                } else {
                    gather_chunk<RED, XB>(ag, a, xr, beg, deg, maxdeg, k0, nkg, rl, q, xrow);
                }
                // edge tiles prefetch the next tile only now: its x fragments
                // are not live across the gather (register budget)
                if (c == nchunk_l - 1) prefetch(tnext, roff_nn);
                if (a.agg_out && !a.agg_in) {
                    int kq = a.K - k0 - 4 * q;
                    asm volatile("" : "+v"(kq));  // per-lane masks stay VGPR selects here
                    const int aoff = (rl * static_cast<int>(a.ld_agg) + k0 + 4 * q) * 4;
#pragma unroll
                    for (int g = 0; g < RT_KC; ++g) {
                        const int mk = lt_mask(16 * g, kq);
                        if (g < nkg) buf_store4(ag[g], ar, ((aoff + 64 * g) & mk) | (kOOB & ~mk), 0, 0);
                    }
                }
                if constexpr (WL_LDS)
                    mfma_chunk_rt<NTW, true>(acc, ag, swl, a.KG, c * RT_KC, nkg, a.NT, lane);
                else
                    mfma_chunk_rt<NTW, false>(acc, ag, a.wl, a.KG, c * RT_KC, nkg, a.NT, lane);
            }
        }

        // ---- epilogue (bias, relu, dropout and the stores)
        const i32x4 orsrc = tile_rsrc(a.out, a.ldo, a.Fo, t, n_rows);
        const i32x4 zr = a.z ? tile_rsrc(a.z, a.ldz, 16 * a.NT1, t, n_rows) : orsrc;
        if (a.epi.drop.thresh == 128u) {  // bit mode (sbias holds 2 b)
            if (a.epi.relu)
                epilogue<NTW, 2, true, VEC>(acc, a, orsrc, zr, sbias, r, rl, q);
            else
                epilogue<NTW, 2, false, VEC>(acc, a, orsrc, zr, sbias, r, rl, q);
        } else if (a.epi.drop.thresh) {
            if (a.epi.relu)
                epilogue<NTW, 1, true, VEC>(acc, a, orsrc, zr, sbias, r, rl, q);
            else
                epilogue<NTW, 1, false, VEC>(acc, a, orsrc, zr, sbias, r, rl, q);
        } else if (a.epi.relu) {
            epilogue<NTW, 0, true, VEC>(acc, a, orsrc, zr, sbias, r, rl, q);
        } else {
            epilogue<NTW, 0, false, VEC>(acc, a, orsrc, zr, sbias, r, rl, q);
        }
    }
}

int g_num_cus[64];

int num_cus() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) return 256;
    if (!g_num_cus[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        g_num_cus[dev] = n;
    }
    return g_num_cus[dev];
}

template <int NTW, int RED, int WLM, bool X3, bool VEC, bool XB, bool W1>
int launch_rt(const RtArgs &a, int n_tiles, size_t lds_bytes, hipStream_t st) {
    auto fn = k_sage_rt<NTW, RED, WLM, X3, VEC, XB, W1>;
    static bool attr_set = false;  // benign race: idempotent
    if (!attr_set) {
        // 160 KiB per CU minus the kernel's static LDS (the tile counter)
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(fn),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 256);
        attr_set = true;
    }
    const int grid = static_cast<int>(
        std::max<int64_t>(1, std::min<int64_t>(num_cus(), ceil_div(n_tiles, RT_WAVES))));
    hipLaunchKernelGGL(fn, dim3(grid), dim3(RT_WAVES * 64), lds_bytes, st, a);
    return launch_status();
}

template <int NTW>
int dispatch_rt(const RtArgs &a, int reduce, bool wl_lds, bool x3, int n_tiles, size_t lds,
                hipStream_t st) {
    // vec: F_out a whole number of 16-column tiles with 16-B aligned rows
    const bool vec = a.vec_out && (a.Fo == a.NT * 16);
    auto by_red = [&](auto red_c) {
        constexpr int RED = decltype(red_c)::value;
        auto go = [&](auto x3_c, auto vec_c, auto xb_c, auto w1_c) {
            constexpr bool X3 = decltype(x3_c)::value, VEC = decltype(vec_c)::value;
            constexpr bool XB = decltype(xb_c)::value, W1 = decltype(w1_c)::value;
            return wl_lds ? launch_rt<NTW, RED, 1, X3, VEC, XB, W1>(a, n_tiles, lds, st)
                          : launch_rt<NTW, RED, 0, X3, VEC, XB, W1>(a, n_tiles, lds, st);
        };
        using T = std::true_type;
        using F = std::false_type;
#if NGNN_RT_FAST_BUILD
        // (kernel-development builds: the fp32 split-bf16 kernels only -- every
        // other layer form returns NGNN_E_SHAPE; minutes less to compile)
        return vec ? go(T{}, T{}, F{}, F{}) : go(T{}, F{}, F{}, F{});
#else
        // one-part images (bf16-exact weights): MEAN / SUM only (the caller checks)
        if constexpr (RED != NGNN_REDUCE_MAX) {
            if (a.w1) {
                if (a.x_bf16) return vec ? go(T{}, T{}, T{}, T{}) : go(T{}, F{}, T{}, T{});
                return vec ? go(T{}, T{}, F{}, T{}) : go(T{}, F{}, F{}, T{});
            }
        }
        if (a.x_bf16) return vec ? go(T{}, T{}, T{}, F{}) : go(T{}, F{}, T{}, F{});  // (x3 checked by the caller)
        if (x3) return vec ? go(T{}, T{}, F{}, F{}) : go(T{}, F{}, F{}, F{});
        return vec ? go(F{}, T{}, F{}, F{}) : go(F{}, F{}, F{}, F{});
#endif
    };
#if NGNN_RT_FAST_BUILD
    return by_red(std::integral_constant<int, NGNN_REDUCE_MEAN>{});
#else
    if (reduce == NGNN_REDUCE_MEAN) return by_red(std::integral_constant<int, NGNN_REDUCE_MEAN>{});
    if (reduce == NGNN_REDUCE_SUM) return by_red(std::integral_constant<int, NGNN_REDUCE_SUM>{});
    return by_red(std::integral_constant<int, NGNN_REDUCE_MAX>{});
#endif
}

// ---- narrow-mode neighbour term: out[d, :Fo] += reduce_{e into d} z[col[e], :Fo]
// for rows d with in-edges below min(n_rows, *n_rows_dev, *n_edge_rows_dev):
// mean/sum of z = x W_l^T (linear, so equal to W_l . mean(x) up to fp32
// rounding).  16 lanes per row (float4 columns), 4 rows per wave, 8
// neighbour rows in flight per lane; per column edge order from 0, then
// / deg for mean.
constexpr int NA_UNR = 8;
template <bool MEAN>
__global__ __launch_bounds__(256) void k_narrow_agg(const float *__restrict__ z, int64_t ldz, int Fo,
                                                    const int32_t *__restrict__ rowptr,
                                                    const int32_t *__restrict__ col, int n_rows,
                                                    const int32_t *__restrict__ n_rows_dev,
                                                    const int32_t *__restrict__ n_edge_dev,
                                                    float *__restrict__ out, int64_t ldo) {
    int nr = n_rows;
    if (n_rows_dev) nr = min(nr, *n_rows_dev);
    if (n_edge_dev) nr = min(nr, *n_edge_dev);
    const int sub = threadIdx.x & 15;
    const int F4 = (Fo + 3) >> 2;
    for (int d = (blockIdx.x * blockDim.x + threadIdx.x) >> 4; d < nr; d += (gridDim.x * blockDim.x) >> 4) {
        const int beg = rowptr[d], end = rowptr[d + 1];
        if (beg == end) continue;
        for (int c4 = sub; c4 < F4; c4 += 16) {
            v4f acc{0.f, 0.f, 0.f, 0.f};
            for (int e = beg; e < end; e += NA_UNR) {
                v4f v[NA_UNR];
#pragma unroll
                for (int u = 0; u < NA_UNR; ++u) {
                    const int ee = min(e + u, end - 1);  // a short batch re-reads its last row
                    v[u] = *reinterpret_cast<const v4f *>(z + static_cast<int64_t>(col[ee]) * ldz + 4 * c4);
                }
#pragma unroll
                for (int u = 0; u < NA_UNR; ++u)
                    if (e + u < end) acc += v[u];
            }
            if (MEAN) acc = acc / static_cast<float>(end - beg);
            float *o = out + static_cast<int64_t>(d) * ldo + 4 * c4;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (4 * c4 + j < Fo) o[j] += acc[j];
        }
    }
}

// ---- GCNConv(normalize=False) aggregation of transformed rows, with the
// layer epilogue: out[d] = act(sum_{e into d} z[col[e]] + b) for EVERY row
// d < min(n_rows, *n_rows_dev) (rows without in-edges: act(b)) -- PyG's
// propagate(lin(x)) (aggr='add', edge order from 0) then + bias
// (convolution.py:29-35).  ReLU and the quad-hash dropout exactly as the
// row-tile epilogue (global column keys, col_base 0).  16 lanes per row,
// float4 columns, 8 neighbour rows in flight per lane.
template <bool VEC>
__global__ __launch_bounds__(256) void k_gcn_agg(const float *__restrict__ z, int64_t ldz, int Fo,
                                                 const int32_t *__restrict__ rowptr,
                                                 const int32_t *__restrict__ col, int n_rows,
                                                 const int32_t *__restrict__ n_rows_dev,
                                                 const float *__restrict__ bias, Epi epi,
                                                 const uint64_t *__restrict__ seed_dev,
                                                 float *__restrict__ out, int64_t ldo) {
    int nr = n_rows;
    if (n_rows_dev) nr = min(nr, *n_rows_dev);
    if (seed_dev) epi.drop.reseed(*seed_dev);
    const int sub = threadIdx.x & 15;
    const int F4 = (Fo + 3) >> 2;
    for (int d = (blockIdx.x * blockDim.x + threadIdx.x) >> 4; d < nr; d += (gridDim.x * blockDim.x) >> 4) {
        const int beg = rowptr[d], end = rowptr[d + 1];
        const uint32_t rk = epi.drop.thresh ? epi.drop.row_key(static_cast<uint32_t>(d)) : 0u;
        for (int c4 = sub; c4 < F4; c4 += 16) {
            v4f acc{0.f, 0.f, 0.f, 0.f};
            for (int e = beg; e < end; e += NA_UNR) {
                v4f v[NA_UNR];
#pragma unroll
                for (int u = 0; u < NA_UNR; ++u) {
                    const int ee = min(e + u, end - 1);
                    v[u] = *reinterpret_cast<const v4f *>(z + static_cast<int64_t>(col[ee]) * ldz + 4 * c4);
                }
#pragma unroll
                for (int u = 0; u < NA_UNR; ++u)
                    if (e + u < end) acc += v[u];
            }
            const uint32_t k4 = epi.drop.thresh ? epi.drop.keep4(rk, static_cast<uint32_t>(c4)) : 0xfu;
            v4f o;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = 4 * c4 + j;
                float y = acc[j] + ((bias && c < Fo) ? bias[c] : 0.0f);
                bool zero = epi.relu && y < 0.0f;  // NaN passes, like torch.relu
                if (epi.drop.thresh) zero = zero || !((k4 >> j) & 1u);
                o[j] = zero ? 0.0f : (epi.drop.thresh ? y * epi.drop.scale : y);
            }
            float *op = out + static_cast<int64_t>(d) * ldo + 4 * c4;
            if (VEC) {
                *reinterpret_cast<v4f *>(op) = o;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (4 * c4 + j < Fo) op[j] = o[j];
            }
        }
    }
}

}  // namespace

// Returns 1 and stores the launch status in *rc when the row-tile kernel
// takes this call, 0 when the shape is outside its envelope (the caller then
// runs the 64-row kernel).  Envelope: no input mask, K % 4 == 0 with 16-B
// aligned rows, the W_r image of one column slice fitting in LDS.  Outputs
// wider than one slice (<= 256 columns, fewer when K is large) run as one
// launch per slice; the packed weights are n-tile major, so a slice is a
// contiguous sub-array.  exact: fp32 MFMA for the root term (else the 3 x
// bf16 split, raw weights only).
int sage_fwd_rowtile(const float *x, int64_t ldx, int64_t K, int64_t n_rows,
                     const int32_t *n_rows_dev, const int32_t *rowptr, const int32_t *col,
                     int reduce, const void *wl_packed, const void *wr_packed, const float *bias,
                     int64_t Fo, float *out, int64_t ldo, int relu, float p_drop, uint64_t seed,
                     const uint64_t *seed_dev, float *agg_out, int64_t ld_agg, hipStream_t st,
                     int *rc, int64_t ldw, void *wl_ws, size_t wl_ws_bytes,
                     const float *const *x_dev, bool exact, float *z, int64_t ldz,
                     const int64_t *xrow, const int64_t *const *xrow_dev, int64_t x_rows,
                     const int32_t *col_x, bool x_bf16, bool w_bf16, bool wl_prepacked) {
    // (with x_dev the run-time address must be 16-B aligned, as torch's are)
    if (K % 4 != 0 || ldx % 4 != 0 || (!x_dev && !aligned(x, 16))) return 0;
    if (ldw && (ldw % 4 != 0 || !aligned(wr_packed, 16) || (wl_packed && !aligned(wl_packed, 16))))
        return 0;
    const bool no_root = wr_packed == nullptr;  // raw weights only (checked by the caller)
    if (agg_out && (ld_agg % 4 != 0 || !aligned(agg_out, 16))) return 0;
    // the gather reads neighbour rows through one resource over all of x
    // (unsigned 32-bit offsets below kOOB); every other operand is addressed
    // per 16-row tile (no size limit)
    const bool indexed = xrow != nullptr || xrow_dev != nullptr;
    // (a graph slot may load materialized batches too: the word then holds 0)
    const int64_t ebytes = x_bf16 ? 2 : 4;
    if ((indexed ? std::max(x_rows, n_rows) : n_rows) * ldx * ebytes > kRangeMax || (indexed && x_rows <= 0))
        return 0;
    const int KG = static_cast<int>(ceil_div(K, 16));
    // X3 root term: C bf16 chunks of 32 + T4 fp32 steps of 4 (tails over 12
    // columns become one zero-padded bf16 chunk)
    // (no root term: the X3 layout with an empty image -- no MFMAs, no LDS)
    const bool x3 = (!exact && ldw > 0) || no_root;
    // bf16 rows: X3 layout only, 8-B aligned rows (ldx a multiple of 4 elements)
    if (x_bf16 && (!x3 || z != nullptr || ldx % 4 != 0)) return 0;
    // narrow mode: one launch computes [x W_r^T | x W_l^T] (2 NT1 tiles) --
    // X3 only, no neighbour term, no saved aggregate, no column slicing
    const bool narrow = z != nullptr;
    if (narrow && (!x3 || !wl_packed || ldz < ceil_div(Fo, 16) * 16 || ldz % 4 != 0 || !aligned(z, 16)))
        return 0;
    int C = static_cast<int>(K / 32), T4 = static_cast<int>(ceil_div(K % 32, 4)), kpad = 0;
    if (T4 > X3_TAIL_MAX) {
        C += 1;
        T4 = 0;
        kpad = 1;
    }
    if (no_root) C = T4 = kpad = 0;
    // bf16-exact weights (NGNN_W_BF16): a one-part image (MEAN / SUM kernels)
    const bool w1 = w_bf16 && x3 && !no_root && reduce != NGNN_REDUCE_MAX;
    // (development builds hold the fp32 split-bf16 MEAN kernels only)
    if (NGNN_RT_FAST_BUILD && (!x3 || x_bf16 || w1 || reduce != NGNN_REDUCE_MEAN)) return 0;
    const size_t frag_kb = static_cast<size_t>(KG) * 64 * sizeof(v4f);  // one fp32 m-tile, all of K
    // one m-tile of the root image: X3 3 parts (1 with w1) x C chunks x 1 KiB + the tail
    const size_t root_kb = x3 ? (static_cast<size_t>((w1 ? 1 : 3) * C) * 64 * 16 +
                                 static_cast<size_t>(T4) * 64 * 4)
                              : frag_kb;
    // (no root term: the slice width is set by the W_l image alone)
    const size_t img_kb = no_root ? frag_kb : root_kb;
    const size_t lds_cap = 160 * 1024 - 1024 - 256;  // minus the bias slice and static LDS
    int ntw_max = 0;
    for (int c : {16, 8, 6, 4, 3, 2})
        if (c <= NGNN_RT_MAXNTW && static_cast<size_t>(c) * img_kb <= lds_cap) {
            ntw_max = c;
            break;
        }
    if (ntw_max == 0) return 0;
    if (narrow && 2 * ceil_div(Fo, 16) > ntw_max) return 0;  // both halves in one image
    const int64_t slice = narrow ? Fo : 16 * static_cast<int64_t>(ntw_max);
    const Dropout drop = make_dropout(p_drop, seed);
    for (int64_t c0 = 0; c0 < Fo; c0 += slice) {
        const int64_t Fo_c = std::min<int64_t>(slice, Fo - c0);
        const int NT1 = static_cast<int>(ceil_div(Fo_c, 16));
        const int NT = narrow ? 2 * NT1 : NT1;
        const int NTW = NT <= 2 ? 2 : NT <= 3 ? 3 : NT <= 4 ? 4 : NT <= 6 ? 6 : NT <= 8 ? 8 : 16;
        const size_t rbytes = static_cast<size_t>(NTW) * root_kb;
        const size_t wbytes = static_cast<size_t>(NTW) * frag_kb;
        const size_t bbytes = static_cast<size_t>(NTW) * 16 * sizeof(float);
        // W_l (fp32) shares the LDS when both fit; otherwise its fragments stream from L2
        const bool has_l = wl_packed != nullptr && !narrow;
        const bool wl_lds = has_l && rbytes + wbytes + bbytes <= lds_cap + 1024;
        const size_t lds = rbytes + (wl_lds ? wbytes : 0) + bbytes;
        const int64_t toff = (c0 / 16) * KG * 64;
        RtArgs a;
        a.x = x;
        a.ldx = ldx;
        a.K = static_cast<int>(K);
        a.KG = KG;
        a.n_rows = static_cast<int>(n_rows);
        a.n_rows_dev = n_rows_dev;
        a.rowptr = rowptr;
        a.col = col;
        // a slice's weights: packed fragments are n-tile major (contiguous
        // sub-array); raw weights are rows [c0, c0 + Fo_c)
        const int64_t woff = ldw ? c0 * ldw / 4 : toff;
        a.wl = has_l ? static_cast<const v4f *>(wl_packed) + woff : nullptr;
        a.wr = no_root ? nullptr : static_cast<const v4f *>(wr_packed) + woff;
        a.wr_raw = (ldw && !no_root) ? static_cast<const float *>(wr_packed) + c0 * ldw : nullptr;
        a.ldw = ldw;
        a.C = C;
        a.T4 = T4;
        a.kpad = kpad;
        if (ldw && has_l && !wl_lds) {
            // raw W_l that must stream from L2: pack it once (all slices) into
            // the caller's workspace -- fragment-ordered 1-KiB wave loads
            if (c0 == 0) {
                if (!wl_ws || wl_ws_bytes < ngnn_pack_weight_bytes(Fo, K)) {
                    *rc = NGNN_E_WORKSPACE;
                    return 1;
                }
                // (NGNN_WL_PREPACKED: the producer packed this step's W_l there)
                const int prc = wl_prepacked ? 0
                                             : ngnn_pack_weight(static_cast<const float *>(wl_packed),
                                                                ldw, Fo, K, wl_ws, st);
                if (prc) {
                    *rc = prc;
                    return 1;
                }
            }
            a.wl = static_cast<const v4f *>(wl_ws) + toff;
        }
        a.NT = NT;
        a.NT1 = NT1;
        a.wz_raw = narrow ? static_cast<const float *>(wl_packed) : nullptr;
        a.z = z;
        a.ldz = ldz;
        a.Fo = static_cast<int>(Fo_c);
        a.out = out + c0;
        a.ldo = ldo;
        a.vec_out = (Fo_c % 4 == 0) && (ldo % 4 == 0) && aligned(out + c0, 16);
        a.agg_out = (c0 == 0 && !narrow) ? agg_out : nullptr;
        a.ld_agg = ld_agg;
        // later column slices read the aggregate the first one saved (the
        // launches are stream-ordered) instead of gathering it again
        a.agg_in = (c0 > 0 && !narrow && has_l) ? agg_out : nullptr;
        a.epi = Epi{bias ? bias + c0 : nullptr, relu, drop, static_cast<int>(c0)};
        a.seed_dev = seed_dev;
        a.x_dev = x_dev;
        a.xrow = xrow;
        a.xrow_dev = xrow_dev;
        a.x_rows = x_rows;
        a.col_x = (xrow || xrow_dev) ? col_x : nullptr;
        a.x_bf16 = x_bf16;
        a.w1 = w1;
        const int n_tiles = static_cast<int>(ceil_div(n_rows, RT_ROWS));
        switch (NTW) {
            case 2: *rc = dispatch_rt<2>(a, reduce, wl_lds, x3, n_tiles, lds, st); break;
            case 3: *rc = dispatch_rt<3>(a, reduce, wl_lds, x3, n_tiles, lds, st); break;
            case 4: *rc = dispatch_rt<4>(a, reduce, wl_lds, x3, n_tiles, lds, st); break;
            case 6: *rc = dispatch_rt<6>(a, reduce, wl_lds, x3, n_tiles, lds, st); break;
            case 8: *rc = dispatch_rt<8>(a, reduce, wl_lds, x3, n_tiles, lds, st); break;
            default: *rc = dispatch_rt<16>(a, reduce, wl_lds, x3, n_tiles, lds, st); break;
        }
        if (*rc) return 1;
    }
    return 1;
}

}  // namespace ngnn

using namespace ngnn;

extern "C" size_t ngnn_sage_fwd_raw_workspace_bytes(int64_t K, int64_t Fo, int64_t n_rows) {
    // a packed W_l (when it cannot sit in LDS), or narrow mode's z rows
    const size_t z = static_cast<size_t>(std::max<int64_t>(n_rows, 0)) * ceil_div(Fo, 16) * 16 *
                     sizeof(float);
    return std::max(ngnn_pack_weight_bytes(Fo, K), z);
}

extern "C" int ngnn_sage_fwd_raw(const float *x, const float *const *x_dev, const int64_t *xrow,
                                 const int64_t *const *xrow_dev, int64_t x_rows, int64_t ldx,
                                 int64_t K, int64_t n_rows, const int32_t *n_rows_dev,
                                 int64_t n_edge_rows, const int32_t *n_edge_rows_dev,
                                 const int32_t *rowptr, const int32_t *col, const int32_t *col_x,
                                 int reduce, const float *wl, const float *wr,
                                 int64_t ldw, const float *bias, int64_t Fo, float *out,
                                 int64_t ldo, int relu, float p_drop, uint64_t seed,
                                 const uint64_t *seed_dev, float *agg_out, int64_t ld_agg, void *ws,
                                 size_t ws_bytes, void *stream) {
    (void)n_edge_rows;  // (row hints of the retired split path; kept for the ABI)
    (void)n_edge_rows_dev;
    const bool exact = (reduce & NGNN_MATH_EXACT_F32) != 0;
    const bool want_narrow = (reduce & NGNN_FWD_NARROW) != 0;
    const bool x_bf16 = (reduce & NGNN_X_BF16) != 0;
    const bool w_bf16 = (reduce & NGNN_W_BF16) != 0;
    const bool wl_prepacked = (reduce & NGNN_WL_PREPACKED) != 0;
    reduce &= ~(NGNN_MATH_EXACT_F32 | NGNN_FWD_NARROW | NGNN_X_BF16 | NGNN_W_BF16 |
                NGNN_WL_PREPACKED);
    // bf16 rows: the split-bf16 root term and the fused path only
    if (x_bf16 && (exact || want_narrow)) return NGNN_E_SHAPE;
    NGNN_RETURN_IF(reduce < NGNN_REDUCE_SUM || reduce > NGNN_REDUCE_MAX, NGNN_E_ARG);
    // wr == NULL: no root term (GCNConv = SAGEConv with W_r = 0: the layer
    // aggregates first, out = act(b + agg(x) W_l^T))
    NGNN_RETURN_IF(K <= 0 || Fo <= 0 || n_rows < 0 || (!wr && !wl), NGNN_E_ARG);
    NGNN_RETURN_IF(!wr && (want_narrow || ldw <= 0), NGNN_E_ARG);
    NGNN_RETURN_IF(wl && !rowptr, NGNN_E_ARG);
    NGNN_RETURN_IF(ldx < K || ldo < Fo || ldw < K, NGNN_E_SHAPE);
    NGNN_RETURN_IF(agg_out && ld_agg < K, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(K) || !fits_i32(n_rows) || !fits_i32(Fo), NGNN_E_RANGE);
    NGNN_RETURN_IF(p_drop < 0.0f || !(p_drop <= 1.0f), NGNN_E_ARG);
    if (n_rows == 0) return NGNN_OK;
    NGNN_RETURN_IF((!x && !x_dev) || !out, NGNN_E_ARG);
    hipStream_t st = as_stream(stream);
    int rc = NGNN_OK;
    // narrow mode (MEAN / SUM): the neighbour term aggregated in the F_out-wide
    // space (z = x W_l^T, then a gather of z), no saved aggregate
    const int64_t ldz = ceil_div(Fo, 16) * 16;
    if (want_narrow && wl && reduce != NGNN_REDUCE_MAX && !agg_out && !relu && !(p_drop > 0.0f) &&
        ws && aligned(ws, 16) &&
        ws_bytes >= static_cast<size_t>(n_rows) * ldz * sizeof(float)) {
        float *z = static_cast<float *>(ws);
        if (sage_fwd_rowtile(x, ldx, K, n_rows, n_rows_dev, rowptr, col, reduce, wl, wr, bias, Fo,
                             out, ldo, relu, p_drop, seed, seed_dev, nullptr, K, st, &rc, ldw,
                             nullptr, 0, x_dev, exact, z, ldz, xrow, xrow_dev, x_rows, col_x, false,
                             w_bf16, false)) {
            if (rc) return rc;
            const int64_t rows = std::max<int64_t>(1, std::min(n_edge_rows, n_rows));
            const unsigned grid = static_cast<unsigned>(
                std::max<int64_t>(1, std::min<int64_t>(4 * num_cus(), ceil_div(rows, 16))));
            if (reduce == NGNN_REDUCE_MEAN)
                hipLaunchKernelGGL(k_narrow_agg<true>, dim3(grid), dim3(256), 0, st, z, ldz,
                                   static_cast<int>(Fo), rowptr, col, static_cast<int>(n_rows),
                                   n_rows_dev, n_edge_rows_dev, out, ldo);
            else
                hipLaunchKernelGGL(k_narrow_agg<false>, dim3(grid), dim3(256), 0, st, z, ldz,
                                   static_cast<int>(Fo), rowptr, col, static_cast<int>(n_rows),
                                   n_rows_dev, n_edge_rows_dev, out, ldo);
            return launch_status();
        }
    }
    if (!sage_fwd_rowtile(x, ldx, K, n_rows, n_rows_dev, rowptr, col, reduce, wl, wr, bias, Fo, out,
                          ldo, relu, p_drop, seed, seed_dev, agg_out, ld_agg, st, &rc, ldw, ws,
                          ws_bytes, x_dev, exact, nullptr, 0, xrow, xrow_dev, x_rows, col_x, x_bf16,
                          w_bf16, wl_prepacked))
        return NGNN_E_SHAPE;  // outside the row-tile envelope: pack + ngnn_sage_fwd
    return rc;
}

extern "C" int ngnn_gcn_agg_fwd(const float *z, int64_t ldz, int64_t Fo, const int32_t *rowptr,
                                const int32_t *col, int64_t n_rows, const int32_t *n_rows_dev,
                                const float *bias, int relu, float p_drop, uint64_t seed,
                                const uint64_t *seed_dev, float *out, int64_t ldo, void *stream) {
    NGNN_RETURN_IF(Fo <= 0 || n_rows < 0 || p_drop < 0.0f || !(p_drop <= 1.0f), NGNN_E_ARG);
    NGNN_RETURN_IF(ldz < ceil_div(Fo, 4) * 4 || ldz % 4 != 0 || ldo < Fo, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(n_rows) || !fits_i32(Fo), NGNN_E_RANGE);
    if (n_rows == 0) return NGNN_OK;
    NGNN_RETURN_IF(!z || !rowptr || !col || !out, NGNN_E_ARG);
    NGNN_RETURN_IF(!aligned(z, 16), NGNN_E_ALIGN);
    const Epi epi{bias, relu, make_dropout(p_drop, seed), 0};
    const unsigned grid = static_cast<unsigned>(
        std::max<int64_t>(1, std::min<int64_t>(8 * num_cus(), ceil_div(n_rows, 16))));
    const bool vec = Fo % 4 == 0 && ldo % 4 == 0 && aligned(out, 16);
    if (vec)
        hipLaunchKernelGGL(k_gcn_agg<true>, dim3(grid), dim3(256), 0, as_stream(stream), z, ldz,
                           static_cast<int>(Fo), rowptr, col, static_cast<int>(n_rows), n_rows_dev,
                           bias, epi, seed_dev, out, ldo);
    else
        hipLaunchKernelGGL(k_gcn_agg<false>, dim3(grid), dim3(256), 0, as_stream(stream), z, ldz,
                           static_cast<int>(Fo), rowptr, col, static_cast<int>(n_rows), n_rows_dev,
                           bias, epi, seed_dev, out, ldo);
    return launch_status();
}
