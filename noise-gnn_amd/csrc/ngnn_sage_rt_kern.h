// k_sage_rt (the row-tile SAGEConv forward kernel) and its launch
// templates, shared by ngnn_sage_rt.hip (host dispatch) and the per-(NTW, RED)
// instantiation units (ngnn_rt_tu.hip).  See ngnn_sage_rt.hip for the design.
#pragma once
#include <cstdlib>
#include <type_traits>

#include "ngnn_device.h"

#ifndef NGNN_RT_WSTREAM_DEPTH
#define NGNN_RT_WSTREAM_DEPTH 2  // (A/B build flag) W_l fragment groups in flight from L2
#endif
#ifndef NGNN_RT_NB_H
#define NGNN_RT_NB_H 4  // (A/B build flag) output tiles per streamed group of the bf16 neighbour term
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
#ifndef NGNN_RT_DBG_CONTIG
#define NGNN_RT_DBG_CONTIG 0  // (diagnostic) output stores at tile-contiguous offsets (wrong layout)
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

}  // namespace

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
    int out_bf16;  // out rows are bf16 (RNE): a bf16 model's hidden activations (VEC only)
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
    // rows with in-edges all lie below min(n_edge, *n_edge_dev) (n_edge_dev may
    // be null); the tiles past it run the root-term-only loop
    int n_edge;
    const int32_t *n_edge_dev;
    // 1: the tiles past the edge-row bound belong to k_root (ngnn_root.hip,
    // launched after this kernel): stop there
    int root_split;
    // non-null: the X3 root image (sw3 + tail, the LDS layout) prebuilt in
    // global memory by k_x3_image -- the prologue copies it by LDS-DMA
    // instead of every workgroup splitting W_r from scattered row reads
    const v4f *img;
    const float *wz_raw;
    float *z;
    int64_t ldz;
    // non-null (one-part W1 layers, W_l streamed from L2): W_l as a bf16
    // image [NT][CL][64] x 16 B for the neighbour term on 16x16x32 bf16 MFMA
    // (k_pack_wl_b16: lane (q, m) holds W_l[16 t + m][32 c + 4 q + j] for j <
    // 4 and [32 c + 16 + 4 q + j - 4] for j >= 4 -- the order of the fp32
    // aggregate fragments ag[2 c], ag[2 c + 1] the lane already holds);
    // CL = ceil(K / 32)
    const void *wlb;
    int CL;
    // non-null: k_x3_image also packs the bf16 W_l image (wlb, all wlb_fo
    // rows) from these raw rows (row stride ldw) -- one launch for both images
    const float *wlb_src;
    int wlb_fo;
    // non-null: k_x3_image also packs the fp32 W_l (ngnn_pack_weight's
    // layout, wlp_fo x K, row stride ldw) into wlp_dst -- the streamed-W_l
    // layers' pack launch folded into the root image's (round 6)
    const float *wlp_src;
    v4f *wlp_dst;
    int wlp_fo;
};

namespace {

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
// the same over 2-byte elements (bf16 rows, ld in elements)
__device__ __forceinline__ i32x4 tile_rsrc2(const void *base, int64_t ld, int cols, int t,
                                            int n_rows) {
    const int left = n_rows - t * 16;
    const uint32_t bytes = left > 16 ? static_cast<uint32_t>((16 * ld + 128) * 2)
                                     : static_cast<uint32_t>(((left - 1) * ld + cols) * 2) * (left > 0);
    return make_rsrc(static_cast<const uint16_t *>(base) + static_cast<int64_t>(t) * 16 * ld, bytes);
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

// neighbour term of one 128-column group on bf16 MFMA (W1 layers: W_l is
// bf16-exact, one part): per 32-deep chunk the lane's fp32 aggregate values
// (ag[2 c], ag[2 c + 1]: columns 32 c + 4 q .. + 3 and 32 c + 16 + 4 q .. + 3
// of its row) split into three bf16 parts (|agg - a1 - a2 - a3| <= 2^-24
// |agg|, split3), three v_mfma_f32_16x16x32_bf16 per output tile against the
// W_l image of the same column order, smallest product first -- the
// fp32-exact 16x16x4 f32 steps this replaces cost 5.3x the MFMA cycles.  The
// image streams from L2 in groups of H output tiles, one group ahead, over
// the chunks without a restart.  Chunks past nkg (columns past K) are
// skipped; their image slots are zero anyway.
template <int NTW>
__device__ __forceinline__ void nb_chunk_b16(v4f (&acc)[NTW], const v4f (&ag)[RT_KC],
                                             const bf16x8 *__restrict__ wlb, int CL, int cc0,
                                             int nkg, int NT, int lane) {
    asm volatile("" : "+s"(NT));
    asm volatile("" : "+s"(CL));
    constexpr int H = NTW % NGNN_RT_NB_H == 0 ? NGNN_RT_NB_H : NTW % 3 == 0 ? 3 : NTW;  // tiles per streamed group
    constexpr int NG = NTW / H;
    constexpr int NS = (RT_KC / 2) * NG;  // steps: (32-chunk, group)
    auto wload = [&](bf16x8 (&w)[H], int s) __attribute__((always_inline)) {
        const int cc = min(cc0 + s / NG, CL - 1);
#pragma unroll
        for (int h = 0; h < H; ++h) {
            const int m = min((s % NG) * H + h, NT - 1);
            w[h] = wlb[(static_cast<int64_t>(m) * CL + cc) * 64 + lane];
        }
    };
    bf16x8 wb[2][H];
    bf16x8 x1, x2, x3;
    wload(wb[0], 0);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int c = s / NG, g = s % NG;
        if (s + 1 < NS) wload(wb[(s + 1) & 1], s + 1);
        if (g == 0) split3<false>(ag[2 * c], ag[2 * c + 1], x1, x2, x3);
        if (2 * c < nkg) {
#pragma unroll
            for (int h = 0; h < H; ++h) {
                const int m = g * H + h;
                v4f t = acc[m];
                t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[s & 1][h], x3, t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[s & 1][h], x2, t, 0, 0, 0);
                acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[s & 1][h], x1, t, 0, 0, 0);
            }
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
            // bf16 rows: all four neighbours' 8-B pieces issued before the
            // first sum (half the registers of fp32 fragments; summed in
            // edge order below, so the result is unchanged)
            i32x2 rb[XB ? 4 : 1][RT_KC];
            if (XB) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int e = e0 + 4 * e4 + j;
                    const int o = lt_mask(e, deg)
                                      ? static_cast<int>(static_cast<uint32_t>(__shfl(cb[j], srcl)) * ld4 + kofs)
                                      : kOOB;
#pragma unroll
                    for (int g = 0; g < RT_KC; ++g) rb[XB ? j : 0][g] = buf_load2i(xr, o + 32 * g, 0, 0);
                }
            }
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
                        v0[g] = bf16x4_to_f32(rb[XB ? j : 0][g]);
                        v1[g] = bf16x4_to_f32(rb[XB ? j + 1 : 0][g]);
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

// epilogue: lane holds output features m*16 + 4q .. +3 of row r; acc already
// holds b + x W^T (the accumulators start from the bias, read from LDS at the
// top of the tile, so the epilogue reads nothing).  Stores go through a
// buffer resource (rows past n_rows are dropped by the range); padded tiles
// (m >= NT) store past the range (dropped, no branch).  VEC:
// F_out a multiple of 16 with 16-B aligned rows -- one 16-B store per m-tile
// at immediate offset 64 m from one per-tile address.  OB: bf16 rows (8-B
// stores).  NAR: narrow mode -- tiles [NT1, NT) are z = x W_l^T rows (their
// bias is 0; a uniform branch per tile m).  The per-tile dispatch picks one
// of these copies once per tile; inside, no branches besides NAR's.
// DM (dropout mode, ngnn_device.h): 0 none; 1 byte mode -- the lane's four
// columns f .. f+3 (f = col_base + 16 m + 4 q, col_base a multiple of 16) are
// one hash quad, pb + 4 m; 2 bit mode (p = 0.5) -- column c is bit c & 31 of
// hash word c >> 5, so two consecutive 16-column tiles share one word and the
// lane's four bits of tile m sit at 16 (gc & 1) + 4 q (gc = the global
// 16-column tile): one shift per tile, then four immediate bit fields.  In
// bit mode the survivor scale 2 is exact (2 acc), and ReLU is an INTEGER max
// with 0 (a pre-activation with the sign bit set -- negative, -0.0 or a
// negative-signed NaN -- gives +0.0; a positive NaN passes), then one AND
// with the keep mask: 3.5 VALU per element.
template <int NTW, int DM, bool RELU, bool VEC, bool OB, bool NAR, bool ODD = false, bool NARF = false>
__device__ __forceinline__ void epilogue(const v4f (&acc)[NTW], const RtArgs &a, i32x4 orsrc,
                                         i32x4 zr, int r, int rl, int q) {
    static_assert(!NAR || (DM == 0 && !RELU && !OB), "narrow: the output layer's plain form");
    static_assert(!OB || VEC, "bf16 rows: whole 16-column tiles");
    // orsrc / zr: the tile's output / z rows (rl = row in the tile); r, the
    // global row, keys the dropout hash
    const uint32_t thresh = a.epi.drop.thresh;
    const float scale = a.epi.drop.scale;
    const uint32_t rk = DM ? a.epi.drop.row_key(static_cast<uint32_t>(r)) : 0u;
    const uint32_t pb = DM == 1 ? rk + static_cast<uint32_t>((a.epi.col_base + 4 * q) >> 2) : 0u;
    const int cb16 = a.epi.col_base >> 4;  // global 16-column tile of m = 0 (uniform)
    uint32_t hw = 0;                       // bit mode: the current hash word
    const int obase = rl * static_cast<int>(a.ldo) * (OB ? 2 : 4) + (OB ? 8 : 16) * q;
    // re-materialised per call: the per-tile-index tests below must not be
    // hoisted out of the tile loop as SGPR lane masks (they spill)
    int NT = a.NT, NT1 = a.NT1;
    asm volatile("" : "+s"(NT));
    asm volatile("" : "+s"(NT1));
    // narrow: z tile m (>= NT1) at zbase + 64 m, the same immediate as out's
    const int zbase = NAR ? rl * static_cast<int>(a.ldz) * 4 + 16 * q - 64 * (NARF ? NTW / 2 : NT1) : 0;
#pragma unroll
    for (int m = 0; m < NTW; ++m) {
        // padded tiles (m >= NT, uniform): the store offset past the range
        // (dropped).  NB the range check covers voffset + imm only, never the
        // scalar soffset -- a "past the range" soffset would still write.
        // (select, then + the tile's immediate: kOOB + 64 m stays past every range)
        const bool live = m < NT;
        // (uniform branch; NARF: NT1 = NTW / 2, compile-time) z rows: 16-B stores, no epilogue
        if (NAR && (NARF ? m >= NTW / 2 : m >= NT1)) {
            buf_store4(acc[m], zr, (live ? zbase : kOOB) + 64 * m, 0, 0);
            continue;
        }
        const int gc = cb16 + m;  // global 16-column tile (uniform)
        // (ODD: cb16 is odd -- the tile parity, hence where a new hash word
        // starts, is compile-time: no branch)
        const int par = (m + (ODD ? 1 : 0)) & 1;  // (a constant after unrolling)
        uint32_t hs = 0;  // bit mode: this lane's four bits of tile m in bits 0..3
        if (DM == 2) {
            if (m == 0 || par == 0) hw = lowbias32(rk + static_cast<uint32_t>(gc >> 1));
            hs = hw >> ((par << 4) + 4 * q);
        }
        const uint32_t h = DM == 1 ? lowbias32(pb + 4u * m) : 0u;
        v4f v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (DM == 2) {
                int yi = __float_as_int(acc[m][j] * 2.0f);
                if (RELU) yi = max(yi, 0);
                v[j] = __int_as_float(yi & bit_mask_at(hs, j));
            } else {
                const float y = acc[m][j];
                // y < 0 (ReLU; NaN passes, like torch.relu) or a dropped column -> 0
                bool zero = RELU && y < 0.0f;
                if (DM == 1) zero = zero || ((h >> (8 * j)) & 0xffu) < thresh;
                v[j] = zero ? 0.0f : (DM == 1 ? y * scale : y);
            }
        }
        if (NGNN_RT_DBG_NOSTORE && v[0] != 1234.5f) continue;
        if (OB) {  // 4 bf16 (hardware RNE), one 8-B store
            typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
            const bf16x2 p0{static_cast<__bf16>(v[0]), static_cast<__bf16>(v[1])};
            const bf16x2 p1{static_cast<__bf16>(v[2]), static_cast<__bf16>(v[3])};
            i32x2 w;
            w.x = __builtin_bit_cast(int, p0);
            w.y = __builtin_bit_cast(int, p1);
            buf_store2i(w, orsrc, (live ? obase : kOOB) + 32 * m, 0, 0);
        } else if (VEC && NGNN_RT_DBG_CONTIG) {  // (diagnostic: tile-contiguous 1-KiB stores)
            buf_store4(v, orsrc, (live ? (rl + 16 * q) * 16 : kOOB) + 1024 * m, 0, 0);
        } else if (VEC) {
            buf_store4(v, orsrc, (live ? obase : kOOB) + 64 * m, 0, 0);
        } else {
            const int f = m * 16 + 4 * q;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                buf_store1(v[j], orsrc, (live && f + j < a.Fo) ? obase + 4 * (16 * m + j) : kOOB, 0, 0);
        }
    }
}

// The split-bf16 root image in LDS: W_r split into three bf16 parts (one
// with W1), one lane fragment (8 consecutive k of one output row) per slot,
// [NP][C][NTW][64] bf16x8, then the fp32 tail [T4][NTW][64]; rows past F_out
// / columns past K are zero.  Image row n: W_r row n (tiles < NT1), W_l row
// n - 16 NT1 (narrow mode's tiles [NT1, NT)), nothing for padded tiles (>= NT)
// or rows past F_out of either half.  All nthreads threads of the workgroup.
template <int NTW, bool W1>
__device__ __forceinline__ void build_x3_image(const RtArgs &a, bf16x8 *sw3, float *swt, int pst,
                                               int nthreads) {
    auto wrow = [&](int n) -> const float * {
        if (n >= 16 * a.NT) return nullptr;
        const bool zt = n >= 16 * a.NT1;
        const int nn = zt ? n - 16 * a.NT1 : n;
        const float *base = zt ? a.wz_raw : a.wr_raw;
        if (nn >= a.Fo || base == nullptr) return nullptr;
        return base + static_cast<int64_t>(nn) * a.ldw;
    };
    // BATCH slots per thread in flight: their global loads issue together
    // (one L2 round trip per batch, not one per slot -- with 256 threads and
    // a 3,072-slot image the one-at-a-time loop cost ~10 us per launch)
    constexpr int BATCH = 8;
    for (int s0 = threadIdx.x; s0 < pst; s0 += nthreads * BATCH) {
        v4f lo[BATCH], hi[BATCH];
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
            const int sl = s0 + u * nthreads;
            const int l = sl & 63, mt = (sl >> 6) % NTW, cc = (sl >> 6) / NTW;
            const int n = mt * 16 + (l & 15), k = 32 * cc + 8 * (l >> 4);
            lo[u] = v4f{0.f, 0.f, 0.f, 0.f};
            hi[u] = v4f{0.f, 0.f, 0.f, 0.f};
            const float *row = sl < pst ? wrow(n) : nullptr;
            if (row) {
                const float *src = row + k;
                if (k + 8 <= a.K) {
                    lo[u] = gload(reinterpret_cast<const v4f *>(src), 0);
                    hi[u] = gload(reinterpret_cast<const v4f *>(src + 4), 0);
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        lo[u][j] = k + j < a.K ? gload(src, j) : 0.0f;
                        hi[u][j] = k + 4 + j < a.K ? gload(src, 4 + j) : 0.0f;
                    }
                }
            }
        }
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
            const int sl = s0 + u * nthreads;
            if (sl >= pst) break;
            bf16x8 p1, p2, p3;
            split3(lo[u], hi[u], p1, p2, p3);
            sw3[sl] = p1;
            if (!W1) {
                sw3[pst + sl] = p2;
                sw3[2 * pst + sl] = p3;
            }
        }
    }
    const int ntail = a.T4 * NTW * 64;
    for (int sl = threadIdx.x; sl < ntail; sl += nthreads) {
        const int l = sl & 63, mt = (sl >> 6) % NTW, st = (sl >> 6) / NTW;
        const int n = mt * 16 + (l & 15), k = 32 * a.C + 4 * st + (l >> 4);
        const float *row = wrow(n);
        swt[sl] = (row && k < a.K) ? row[k] : 0.0f;
    }
}

// LDS-DMA copy of a prebuilt image into LDS: the bf16 parts (nv v4f, a
// multiple of 64: one 1-KiB wave-instruction per 64) and the fp32 tail (nt
// floats, a multiple of 64: 256-B dword pieces) right behind them, every
// wave's copies in flight at once (the caller waits vmcnt(0) and barriers)
__device__ __forceinline__ void dma_image(v4f *dst, const v4f *src, int nv, int nt, int nwaves) {
    const int wv = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int ln = threadIdx.x & 63;
    for (int c = wv; c < nv / 64; c += nwaves)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(src + c * 64 + ln),
                                         (__attribute__((address_space(3))) void *)(dst + c * 64), 16, 0, 0);
    const float *ts = reinterpret_cast<const float *>(src + nv);
    float *td = reinterpret_cast<float *>(dst + nv);
    for (int c = wv; c < nt / 64; c += nwaves)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(ts + c * 64 + ln),
                                         (__attribute__((address_space(3))) void *)(td + c * 64), 4, 0, 0);
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
        if (X3 && a.img) dma_image(lds, a.img, NP * pst, a.T4 * NTW * 64, RT_WAVES);
        else if (X3) build_x3_image<NTW, W1>(a, sw3, swt, pst, RT_WAVES * 64);
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
        if (X3 && a.img) __builtin_amdgcn_s_waitcnt(0);  // (the image's LDS-DMAs landed)
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
        // (the accumulators' initial value; 0 past F_out and on narrow z tiles)
        for (int i = threadIdx.x; i < NTW * 16; i += RT_WAVES * 64)
            sbias[i] = (a.epi.bias && i < a.Fo) ? a.epi.bias[i] : 0.0f;
    }
    __syncthreads();
#ifdef NGNN_DBG_PROLOGUE_ONLY
    if (a.K != 1234567) return;  // (diagnostic: the image build alone)
#endif

    const int wave = wv;
    int n_rows = a.n_rows;
    if (a.n_rows_dev) n_rows = min(n_rows, *a.n_rows_dev);
    n_rows = __builtin_amdgcn_readfirstlane(n_rows);  // (provably uniform: scalar resources)
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
    auto claim = [&]() __attribute__((always_inline)) -> int {
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
    auto row_off = [&](int rr) __attribute__((always_inline)) -> uint32_t {
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
    auto lane_ids = [&](int &lane_, int &q_, int &rl_) __attribute__((always_inline)) {
        int l = static_cast<int>(threadIdx.x) & 63;
        asm volatile("" : "+v"(l));
        lane_ = l;
        q_ = l >> 4;
        rl_ = l & 15;
    };
    auto prefetch = [&](int tn, uint32_t roff_tn) __attribute__((always_inline)) {
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
    // ---- the tile epilogue: one branch-free copy per tile form (uniform
    // dispatch); acc holds b + x W_r^T (+ agg W_l^T)
    // narrow mode (the output layer: split-bf16, W_l not a neighbour term);
    // bf16 hidden rows (a bf16 model's layers: one-part weight images)
    constexpr bool CAN_NAR = X3 && WLM == 0 && RED != NGNN_REDUCE_MAX;
    constexpr bool CAN_OB = W1 && VEC;
    auto tile_epilogue = [&](const v4f (&acc)[NTW], int t, int r, int rl, int q) __attribute__((always_inline)) {
        const i32x4 orsrc = a.out_bf16 ? tile_rsrc2(a.out, a.ldo, a.Fo, t, n_rows)
                                       : tile_rsrc(a.out, a.ldo, a.Fo, t, n_rows);
        const i32x4 zr = a.z ? tile_rsrc(a.z, a.ldz, 16 * a.NT1, t, n_rows) : orsrc;
        // one branch-free epilogue copy per tile form (uniform dispatch)
        auto epi = [&](auto dm_c, auto relu_c, auto ob_c, auto nar_c) __attribute__((always_inline)) {
            constexpr int DMv = decltype(dm_c)::value;
            constexpr bool RELUv = decltype(relu_c)::value, OBv = decltype(ob_c)::value;
            constexpr bool NARv = decltype(nar_c)::value;
            if (DMv == 2 && ((a.epi.col_base >> 4) & 1))
                epilogue<NTW, DMv, RELUv, VEC, OBv, NARv, true>(acc, a, orsrc, zr, r, rl, q);
            else
                epilogue<NTW, DMv, RELUv, VEC, OBv, NARv, false>(acc, a, orsrc, zr, r, rl, q);
        };
        using T = std::true_type;
        using F = std::false_type;
        using D0 = std::integral_constant<int, 0>;
        using D1 = std::integral_constant<int, 1>;
        using D2 = std::integral_constant<int, 2>;
        auto by_drop = [&](auto ob_c) __attribute__((always_inline)) {
            if (a.epi.drop.thresh == 128u) {  // bit mode
                if (a.epi.relu) epi(D2{}, T{}, ob_c, F{});
                else epi(D2{}, F{}, ob_c, F{});
            } else if (a.epi.drop.thresh) {
                if (a.epi.relu) epi(D1{}, T{}, ob_c, F{});
                else epi(D1{}, F{}, ob_c, F{});
            } else if (a.epi.relu) {
                epi(D0{}, T{}, ob_c, F{});
            } else {
                epi(D0{}, F{}, ob_c, F{});
            }
        };
        if (CAN_NAR && a.NT1 < a.NT) {
            if constexpr (CAN_NAR) epi(D0{}, F{}, F{}, T{});
        } else if (CAN_OB && a.out_bf16) {
            if constexpr (CAN_OB) by_drop(T{});
        } else {
            by_drop(F{});
        }
    };
    // the accumulators start from the bias (one LDS read per output tile,
    // one wait): b + x W_r^T (+ agg W_l^T), no bias add in the epilogue
    auto init_acc = [&](v4f (&acc)[NTW], int q) __attribute__((always_inline)) {
#pragma unroll
        for (int m = 0; m < NTW; ++m) acc[m] = *reinterpret_cast<const v4f *>(sbias + 16 * m + 4 * q);
    };
    // X3 fp32 tail steps (the K % 32 columns past the bf16 chunks): every
    // W value of a step read from LDS before its MFMAs (one wait, not one per
    // pair of output tiles)
    auto tail_mfma = [&](v4f (&acc)[NTW], const float (&xt)[X3_TAIL_MAX], int q, int lane) __attribute__((always_inline)) {
#pragma unroll
        for (int s2 = 0; s2 < X3_TAIL_MAX; ++s2) {
            if (s2 < a.T4) {
                float wt[NTW];
#pragma unroll
                for (int m = 0; m < NTW; ++m) wt[m] = swt[(s2 * NTW + m) * 64 + lane];
                const float xv = __int_as_float(__float_as_int(xt[s2]) & lt_mask(32 * a.C + 4 * s2 + q, a.K));
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int m = 0; m < NTW; ++m)
                    acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(wt[m], xv, acc[m], 0, 0, 0);
            }
        }
    };
    // tiles from t2 on have no in-edges (rows >= the block's edge-row bound,
    // NeighborLoader's order): phase 2 below, a root-term-only loop (X3)
    // phase 2's epilogue form is fixed per launch (its loop holds ONE
    // straight-line epilogue: with the per-tile form dispatch inside the loop
    // the compiler's waits at the tile head stopped counting the previous
    // tile's stores as younger and drained them every tile).  Forms:
    // 1 bit-mode dropout + ReLU, 2 ReLU, 3 plain, 4 narrow; +4: bf16 rows.
    // Other forms (byte-mode dropout, odd column slices) run in phase 1.
    int p2form = 0;
    if (CAN_NAR && a.NT1 < a.NT) {
        // (phase 2's narrow epilogue splits out / z tiles at NTW / 2)
        if (a.NT == NTW && 2 * a.NT1 == NTW) p2form = 4;
    } else {
        const bool odd = (a.epi.col_base >> 4) & 1;
        if (a.epi.drop.thresh == 128u && a.epi.relu && !odd) p2form = 1;
        else if (a.epi.drop.thresh == 0u && a.epi.relu) p2form = 2;
        else if (a.epi.drop.thresh == 0u && !a.epi.relu) p2form = 3;
        if (p2form && CAN_OB && a.out_bf16) p2form = p2form == 3 ? 0 : p2form + 4;
    }
    int t2 = n_tiles;
    if (X3 && !NGNN_RT_STATIC && ((p2form && nchunk <= 2) || a.root_split)) {  // (phase 2 covers 1 or 2 chunks)
        int ne = have_l ? a.n_edge : 0;  // (no neighbour term in the kernel: every tile)
        if (a.n_edge_dev) ne = min(ne, *a.n_edge_dev);
        t2 = __builtin_amdgcn_readfirstlane(min(n_tiles, (max(ne, 0) + RT_ROWS - 1) / RT_ROWS));
    }
    for (; t < t2; t = tnext, ++kt) {
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
        // the accumulators start from the bias (one LDS read per output tile,
        // one wait): b + x W_r^T (+ agg W_l^T), no bias add in the epilogue
        v4f acc[NTW];
        init_acc(acc, q);
        // (X3: the tail first, while the prefetched tail values are still this tile's)
        if (X3) tail_mfma(acc, xtn, q, lane);

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
                if constexpr (WL_LDS) {
                    mfma_chunk_rt<NTW, true>(acc, ag, swl, a.KG, c * RT_KC, nkg, a.NT, lane);
                } else if constexpr (W1) {  // (the host always provides the bf16 image here)
                    nb_chunk_b16<NTW>(acc, ag, static_cast<const bf16x8 *>(a.wlb), a.CL, 4 * c, nkg, a.NT, lane);
                } else {
                    mfma_chunk_rt<NTW, false>(acc, ag, a.wl, a.KG, c * RT_KC, nkg, a.NT, lane);
                }
            }
        }

        // ---- epilogue (relu, dropout and the stores; the bias is in acc)
        tile_epilogue(acc, t, r, rl, q);
    }

    if (a.root_split) return;  // (k_root runs the rest)

    // ---- phase 2 (X3): the tiles without in-edges.  The same tail, root
    // term and epilogue, with the x fragments ping-ponged between two
    // register sets by STEP (one 128-column chunk of one tile): step s runs on
    // set s % 2 while step s + 1 (the tile's next chunk, or the next tile's
    // first) loads into the other.  The chunk count is a compile-time NCH (1:
    // K <= 140, 2: K <= 268; wider layers stay in phase 1) and the loop body
    // spans a whole number of steps per set (2 tiles for NCH = 1, 1 for 2), so
    // every step's set and position is fixed: no register copy, and the wait
    // for a tile's prefetched fragments counts the previous tile's 16 output
    // stores as younger (no store drain per tile).  With phase 1's one
    // loop-carried set the compiler copied the prefetch into it -- waiting
    // for it -- right before every epilogue.
    if constexpr (X3 && !NGNN_RT_STATIC) {
        auto phase2 = [&](auto nch_c, auto form_c) __attribute__((always_inline)) {
            constexpr int NCH = decltype(nch_c)::value;
            constexpr int FORM = decltype(form_c)::value;
            constexpr int FB = FORM > 4 ? FORM - 4 : FORM;  // the form without bf16 rows
            constexpr int DM = FB == 1 ? 2 : 0;
            constexpr bool RELU = FB == 1 || FB == 2, OB = FORM > 4, NAR = FB == 4;
            constexpr int TPB = (NCH % 2) ? 2 : 1;  // tiles per loop body
            v4f xb[RT_KC];
            float xtb[X3_TAIL_MAX] = {0.f, 0.f, 0.f};
#pragma unroll
            for (int g = 0; g < RT_KC; ++g) xb[g] = v4f{0.f, 0.f, 0.f, 0.f};
            // settle tile t's fragments (in flight from phase 1's prefetch, or
            // the first one): a wave entering here straight from the start
            // has no stores behind them, and the compiler's wait at a loop
            // head takes the fewest younger memory ops over the entry paths
#pragma unroll
            for (int g = 0; g < RT_KC; ++g) asm volatile("" : "+v"(xn[g]));
#pragma unroll
            for (int s2 = 0; s2 < X3_TAIL_MAX; ++s2) asm volatile("" : "+v"(xtn[s2]));
            uint32_t roff = roff_n;  // tile t's row offset
            v4f acc[NTW];
            // tile u of the loop body (compile-time u: every step's register
            // set is fixed); false when the wave has no tiles left
            auto one_tile = [&](auto u_c) __attribute__((always_inline)) -> bool {
                constexpr int U = decltype(u_c)::value;
                int lane, q, rl;
                lane_ids(lane, q, rl);
                const int tn = claim();
                const uint32_t roff_tn = row_off(tn * RT_ROWS + rl);
                init_acc(acc, q);
                if constexpr ((U * NCH) % 2 == 0) tail_mfma(acc, xtn, q, lane);
                else tail_mfma(acc, xtb, q, lane);
                const int kq8 = a.K - (32 * (a.C - 1) + 8 * q);
                auto chunk = [&](auto c_c, v4f (&xcur)[RT_KC], v4f (&xnxt)[RT_KC],
                                 float (&xtnxt)[X3_TAIL_MAX]) __attribute__((always_inline)) {
                    constexpr int C_ = decltype(c_c)::value;
                    if constexpr (C_ + 1 < NCH) {
                        load_x<true, XB>(xnxt, xr, roff, (C_ + 1) * RT_KC * 16, q);
                    } else {  // the next tile's chunk 0 and tail (past the end: reads 0)
                        load_x<true, XB>(xnxt, xr, roff_tn, 0, q);
                        load_xt<XB>(xtnxt, a, xr, roff_tn, q);
                    }
                    mfma_group_x3<NTW, XB, W1>(acc, xcur, sw3, pst, 4 * C_, min(4, a.C - 4 * C_),
                                               a.kpad && C_ == NCH - 1, kq8, lane);
                };
                using I0 = std::integral_constant<int, 0>;
                using I1 = std::integral_constant<int, 1>;
                // step s = U NCH + c runs on set s % 2 (xn even, xb odd)
                if constexpr ((U * NCH) % 2 == 0) chunk(I0{}, xn, xb, xtb);
                else chunk(I0{}, xb, xn, xtn);
                if constexpr (NCH == 2) {
                    if constexpr ((U * NCH + 1) % 2 == 0) chunk(I1{}, xn, xb, xtb);
                    else chunk(I1{}, xb, xn, xtn);
                }
                {
                    const i32x4 orsrc = OB ? tile_rsrc2(a.out, a.ldo, a.Fo, t, n_rows)
                                           : tile_rsrc(a.out, a.ldo, a.Fo, t, n_rows);
                    const i32x4 zr = NAR ? tile_rsrc(a.z, a.ldz, 16 * a.NT1, t, n_rows) : orsrc;
                    epilogue<NTW, DM, RELU, VEC, OB, NAR, false, NAR>(acc, a, orsrc, zr, t * RT_ROWS + rl, rl, q);
                }
                t = tn;
                roff = roff_tn;
                return t < n_tiles;
            };
            while (one_tile(std::integral_constant<int, 0>{})) {
                if constexpr (TPB == 2) {
                    if (!one_tile(std::integral_constant<int, 1>{})) break;
                }
            }
        };
        auto run = [&](auto form_c) __attribute__((always_inline)) {
            if (nchunk == 1) phase2(std::integral_constant<int, 1>{}, form_c);
            else phase2(std::integral_constant<int, 2>{}, form_c);
        };
        if (t < n_tiles) {  // (p2form != 0: t2 < n_tiles only then)
            using IC1 = std::integral_constant<int, 1>;
            using IC2 = std::integral_constant<int, 2>;
            using IC3 = std::integral_constant<int, 3>;
            if (p2form == 1) run(IC1{});
            else if (p2form == 2) run(IC2{});
            else if (p2form == 3) run(IC3{});
            else if (CAN_NAR && p2form == 4) {
                if constexpr (CAN_NAR) run(std::integral_constant<int, 4>{});
            } else if (CAN_OB && p2form == 5) {
                if constexpr (CAN_OB) run(std::integral_constant<int, 5>{});
            } else if (CAN_OB && p2form == 6) {
                if constexpr (CAN_OB) run(std::integral_constant<int, 6>{});
            }
        }
    }
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

template <int NTW, int RED>
int dispatch_rt_red(const RtArgs &a, bool wl_lds, bool x3, int n_tiles, size_t lds, hipStream_t st) {
    // vec: F_out a whole number of 16-column tiles with 16-B aligned rows
    const bool vec = a.vec_out && (a.Fo == a.NT * 16);
    auto go = [&](auto x3_c, auto vec_c, auto xb_c, auto w1_c) {
        constexpr bool X3 = decltype(x3_c)::value, VEC = decltype(vec_c)::value;
        constexpr bool XB = decltype(xb_c)::value, W1 = decltype(w1_c)::value;
        return wl_lds ? launch_rt<NTW, RED, 1, X3, VEC, XB, W1>(a, n_tiles, lds, st)
                      : launch_rt<NTW, RED, 0, X3, VEC, XB, W1>(a, n_tiles, lds, st);
    };
    using T = std::true_type;
    using F = std::false_type;
#if NGNN_RT_FAST_BUILD
    // (kernel-development builds: the fp32 split-bf16 MEAN kernels only --
    // sage_fwd_rowtile declines every other layer form; minutes less to compile)
    if constexpr (RED != NGNN_REDUCE_MEAN) {
        return NGNN_E_SHAPE;
    } else {
        return vec ? go(T{}, T{}, F{}, F{}) : go(T{}, F{}, F{}, F{});
    }
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
}

}  // namespace

// One translation unit per (NTW, RED) instantiates the kernels of that pair
// (ngnn_rt_tu.hip, built 18 times by the Makefile: parallel compiles of the
// ~300 k_sage_rt variants); sage_fwd_rowtile dispatches through these.
#define NGNN_RT_FOR_EACH(X) \
    X(2, 0) X(2, 1) X(2, 2) X(3, 0) X(3, 1) X(3, 2) X(4, 0) X(4, 1) X(4, 2) \
    X(6, 0) X(6, 1) X(6, 2) X(8, 0) X(8, 1) X(8, 2) X(16, 0) X(16, 1) X(16, 2)
// k_root (ngnn_root.hip): the tiles past the edge-row bound on the
// one-wave-per-SIMD root-term kernel; NGNN_E_SHAPE when no instantiation
// covers (NTW, C, T4, the epilogue form, bf16 flags) -- nothing launched
int launch_root(const RtArgs &a, int ntw, int form, bool vec, hipStream_t st, bool dry = false);
// the epilogue form of a launch (1 bit-mode dropout + ReLU, 2 ReLU, 3 plain,
// 4 narrow, 5 / 6: 1 / 2 with bf16 rows), 0 for forms without a
// root-term-only loop
int rt_form(const RtArgs &a, int ntw, bool vec);
// bytes of a slice's prebuilt X3 image (ngnn_root.hip) and its build launch
size_t x3_image_bytes(int ntw, int C, int T4, bool w1);
int build_image(RtArgs &a, int ntw, void *dst, hipStream_t st);
#define NGNN_RT_FN(N, R) dispatch_rt_n##N##_r##R
#define NGNN_RT_DECLARE(N, R) \
    int NGNN_RT_FN(N, R)(const RtArgs &a, bool wl_lds, bool x3, int n_tiles, size_t lds, hipStream_t st);
NGNN_RT_FOR_EACH(NGNN_RT_DECLARE)

}  // namespace ngnn
