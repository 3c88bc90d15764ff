// Two-layer SAGE forward of the headline shape as weight-stationary kernels
// (DESIGN.md section 5b): SAGE(K0 -> 256 -> F1), mean / sum, the output layer
// in the narrow form, one NeighborLoader block -- sage.py:33-39 for L = 2:
//
//     h   = dropout(relu(b0 + x W_r0^T + [deg > 0] agg(x) W_l0^T))
//     out = b1 + h W_r1^T + [deg > 0] agg(h) W_l1^T
//
// Why a new decomposition.  The row-tile kernels hold one layer's weights in
// LDS: layer 0's split image (148 KiB) and layer 1's (144 KiB) cannot be
// resident together in the 160 KiB, so layer 0 wrote h (153 k x 256 fp32,
// 157 MB) and layer 1 re-read all of it to project it to 47 + 47 columns.
// Here the weights live in the REGISTER file (512 KiB per CU, 3.2x the LDS):
// each of a workgroup's 8 waves owns 32 of layer 0's 256 output columns and
// keeps its slice of W_r0 and of [W_r1 | W_l1] (the matching 32 rows of
// layer 1's K) in VGPRs for the whole launch.  A 16-row tile of x flows
// through the workgroup: every wave computes its 32 columns of h, applies
// bias / ReLU / dropout, multiplies them by its layer-1 slice and writes a
// partial [16 x 96] of (out | z) to LDS; after one barrier the 8 partials are
// summed in fixed order into out = b1 + h W_r1^T and z = h W_l1^T.  h leaves
// the chip only for the rows the backward reads (< R', the slot's device
// bound; every row when the caller does not know it).
//
// Arithmetic (H2): both operands of every product are
// split into two fp16 parts after a power-of-two scaling (rows of x / h by
// their own max, each weight matrix by its max: max |v| 2^e in [2^14, 2^15)),
// v 2^e = p1 + p2 + r with |r| <= 2^-22 |v 2^e| (subnormal p2: an absolute
// 2^-25 of the scaled unit).  Three fp16 MFMA products per 32-deep chunk
// (p2 p1', p1 p2', p1 p1', each exact in fp32, accumulated in fp32): the
// dropped terms are <= ~3 2^-22 relative per product -- inside the fp32
// parity bars (outputs 1e-5) with half the MFMAs of the 3 x bf16 split.  The
// accumulators are unscaled with v_ldexp (exact).
//
// Three launches, all on the caller's stream:
//   k_prep2    the weight images (fp16 parts in fragment order) and the
//              per-matrix exponents; one workgroup per matrix;
//   k_edge_nb  rows with in-edges (NeighborLoader numbers them first): the
//              neighbour aggregate in edge order (bit-identical to
//              ngnn_seg_agg_fwd; it is the backward's saved aggregate), then
//              nb = agg W_l0^T on MFMA with W_l0's image in LDS;
//   k_fwd2     every row: layer 0's root term + nb + epilogue, layer 1's
//              products, the cross-wave sum; then k_narrow_agg (ngnn_sage_rt.hip)
//              adds mean_j z_j to the rows with in-edges.
#include <algorithm>
#include <type_traits>

#include "ngnn_device.h"

namespace ngnn {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));

constexpr int F2_WAVES = 8;    // workgroup: 8 waves x 32 hidden columns = 256
constexpr int F2_HID = 256;    // hidden width of the fused shape
constexpr int F2_ROWS = 16;    // rows per tile (one MFMA n-block)
constexpr int F2_NB = 4;       // neighbour rows in flight per lane (k_edge_nb)
constexpr int kOOB2 = static_cast<int>(0xF0000000u);  // past every buffer range

// e with max|v| 2^e in [2^14, 2^15) (0 -> 15; inf / NaN rows stay inf / NaN)
__device__ __forceinline__ int h2_exp(float amax) { return 15 - __builtin_amdgcn_frexp_expf(amax); }

// two fp16 parts (round to nearest even) of 8 scaled values
__device__ __forceinline__ void h2_split(v4f a, v4f b, half8 &p1, half8 &p2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float v = j < 4 ? a[j] : b[j - 4];
        const _Float16 h = static_cast<_Float16>(v);
        p1[j] = h;
        p2[j] = static_cast<_Float16>(v - static_cast<float>(h));
    }
}

__device__ __forceinline__ v4f ldexp4(v4f v, int e) {
    v4f o;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = __builtin_amdgcn_ldexpf(v[i], e);
    return o;
}

__device__ __forceinline__ float amax4(v4f v) {
    return fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
}

// cross-lane max of non-negative floats (their bit patterns order as ints),
// on VALU only (no LDS round trip): DPP inside a 16-lane row, the gfx950
// permlane swaps across rows
__device__ __forceinline__ float max_xor16(float v) {  // lanes l and l ^ 16
    const int x = __float_as_int(v);
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return __int_as_float(max(static_cast<int>(r[0]), static_cast<int>(r[1])));
}
__device__ __forceinline__ float max_xor32(float v) {  // lanes l and l ^ 32
    const int x = __float_as_int(v);
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return __int_as_float(max(static_cast<int>(r[0]), static_cast<int>(r[1])));
}
__device__ __forceinline__ float max_row16(float v) {  // all 16 lanes of the row
    int x = __float_as_int(v);
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false));  // row_half_mirror
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, false));  // row_mirror
    return __int_as_float(x);
}

// three-product H2 MFMA: acc += (a1 + a2)(b1 + b2) - a2 b2, smallest first
__device__ __forceinline__ v4f mfma_h2(half8 a1, half8 a2, half8 b1, half8 b2, v4f acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2, b1, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b2, acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b1, acc, 0, 0, 0);
}

// an LDS-only workgroup barrier: the LDS traffic before it has landed, the
// vector-memory traffic (prefetched rows, output stores) stays in flight --
// __syncthreads() would also drain vmcnt.  The asm's memory clobber keeps
// the compiler from moving memory accesses across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ---------------------------------------------------------------- k_prep2
struct P2Args {
    const float *wr0, *wl0;  // [256, K0], row stride ldw0
    int64_t ldw0;
    int K0, C0;
    const float *wr1, *wl1;  // [F1, 256], row stride ldw1
    int64_t ldw1;
    int F1, NT1;
    half8 *img_r0;  // k_fwd2: [8 w][2 mt][C0][2 p][64]
    half8 *img_l0;  // k_edge_nb: [16 mt][C0][2 p][64] (its LDS image)
    half8 *img_1;   // k_fwd2: [8 w][2 NT1][2 p][64]
    int *exps;      // [0] W_r0, [1] W_l0, [2] [W_r1 | W_l1]
};

// blockIdx.y: 0 W_r0, 1 W_l0, 2 layer 1.  Every block reduces its matrix's
// max |w| itself (16-B loads, all in flight: ~100 KB per matrix from L2) --
// no cross-block hand-off -- then writes its share of the image slots (8
// values of one lane, both parts).
constexpr int P2_THREADS = 256;
constexpr int P2_U = 32;  // float4 loads per thread for the max: 32 x 256 = 256 x 128 / 4 (K0 <= 128)
__global__ __launch_bounds__(P2_THREADS) void k_prep2(P2Args a) {
    __shared__ float sred[P2_THREADS / 64];
    const int mat = blockIdx.y;
    float m = 0.0f;
    {
        // the matrix as float4 quads (rows are 16-B aligned: K0 and ldw % 4 == 0)
        const int q0 = mat < 2 ? a.K0 / 4 : F2_HID / 4;  // quads per row
        const int nr = mat < 2 ? F2_HID : 2 * a.F1;
        const int nq = nr * q0;
        v4f t[P2_U];
#pragma unroll
        for (int u = 0; u < P2_U; ++u) {
            const int i = u * P2_THREADS + static_cast<int>(threadIdx.x);
            const int rr = i / q0, c = i - rr * q0;
            const float *row;
            if (mat < 2) row = (mat == 0 ? a.wr0 : a.wl0) + static_cast<int64_t>(min(rr, F2_HID - 1)) * a.ldw0;
            else {
                const int z = rr >= a.F1;
                row = (z ? a.wl1 : a.wr1) + static_cast<int64_t>(min(rr - z * a.F1, a.F1 - 1)) * a.ldw1;
            }
            t[u] = i < nq ? *reinterpret_cast<const v4f *>(row + 4 * c) : v4f{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < P2_U; ++u) m = fmaxf(m, amax4(t[u]));
    }
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6] = m;
    __syncthreads();
    m = 0.0f;
#pragma unroll
    for (int i = 0; i < P2_THREADS / 64; ++i) m = fmaxf(m, sred[i]);
    const int e = h2_exp(m);
    if (threadIdx.x == 0 && blockIdx.x == 0) a.exps[mat] = e;
    const int C0 = a.C0, MT1 = 2 * a.NT1;
    const int nslot = mat == 0 ? F2_WAVES * 2 * C0 * 64 : mat == 1 ? (F2_HID / 16) * C0 * 64 : F2_WAVES * MT1 * 64;
    for (int s = blockIdx.x * P2_THREADS + threadIdx.x; s < nslot; s += gridDim.x * P2_THREADS) {
        const int l = s & 63, f = s >> 6, m16 = l & 15, q = l >> 4;
        float v[8];
        int dst;
        half8 *img;
        if (mat < 2) {
            int n, c;
            if (mat == 0) {  // f = (w 2 + mt) C0 + c
                c = f % C0;
                const int wm = f / C0;  // w 2 + mt
                n = 16 * wm + m16;      // = 32 w + 16 mt + m16
            } else {  // f = mt C0 + c
                c = f % C0;
                n = 16 * (f / C0) + m16;
            }
            const float *w = (mat == 0 ? a.wr0 : a.wl0) + static_cast<int64_t>(n) * a.ldw0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = 32 * c + 8 * q + j;
                v[j] = k < a.K0 ? w[k] : 0.0f;
            }
            dst = f * 2;
            img = mat == 0 ? a.img_r0 : a.img_l0;
        } else {  // f = w MT1 + mt1; k order of the h fragment: 4q + j, 16 + 4q + j - 4
            const int w = f / MT1, mt1 = f - w * MT1;
            const int zt = mt1 >= a.NT1;
            const int o = 16 * (mt1 - zt * a.NT1) + m16;
            const float *row = (zt ? a.wl1 : a.wr1) + static_cast<int64_t>(o) * a.ldw1;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = 32 * w + (j < 4 ? 4 * q + j : 16 + 4 * q + j - 4);
                v[j] = o < a.F1 ? row[k] : 0.0f;
            }
            dst = f * 2;
            img = a.img_1;
        }
        v4f lo{v[0], v[1], v[2], v[3]}, hi{v[4], v[5], v[6], v[7]};
        half8 p1, p2;
        h2_split(ldexp4(lo, e), ldexp4(hi, e), p1, p2);
        img[dst * 64 + l] = p1;
        img[(dst + 1) * 64 + l] = p2;
    }
}

// ---------------------------------------------------------------- k_edge_nb
struct G2Args {
    const float *x;
    const float *const *x_dev;  // non-null: x's address read at run time (graph slot)
    int64_t ldx;
    int K0;
    int n_rows;
    const int32_t *n_rows_dev;
    int n_edge;
    const int32_t *n_edge_dev;
    const int32_t *rowptr, *col;
    // fused x[n_id] gather: x is the feature table (x_rows rows) and col_x =
    // n_id[col] (the slot load writes it); null: x holds the block's rows
    const int32_t *col_x;
    int64_t x_rows;
    int mean;
    const half8 *img_l0;
    const int *exps;
    float *agg;  // saved aggregate [>= rows of the edge tiles, ld_agg]
    int64_t ld_agg;
    float *nb;   // [>= rows of the edge tiles, 256]
    int64_t cap_rows;  // rows of agg / nb
};

// One wave per 16-row tile of the rows with in-edges.  Lane (rl, q) gathers
// columns 32 c + 8 q .. + 7 (c < C0) of its row's neighbours -- already the
// B-fragment layout of the MFMA -- F2_NB neighbours per round trip, summed in
// edge order from +0.0 (padded slots read 0), / max(deg, 1) for mean: the fp32
// sequence of ngnn_seg_agg_fwd.  Then nb = agg W_l0^T (16 m-tiles, W_l0's
// image in LDS), unscaled, 16-B stores.
template <int C0>
__global__ __launch_bounds__(F2_WAVES * 64) void k_edge_nb(G2Args a) {
    extern __shared__ __attribute__((aligned(16))) half8 simg[];  // [16][C0][2][64]
    constexpr int NFR = (F2_HID / 16) * C0 * 2;
    const int wv = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int ln = threadIdx.x & 63;
    for (int f = wv; f < NFR; f += F2_WAVES)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(a.img_l0 + f * 64 + ln),
                                         (__attribute__((address_space(3))) void *)(simg + f * 64), 16, 0, 0);
    int n_rows = a.n_rows;
    if (a.n_rows_dev) n_rows = min(n_rows, *a.n_rows_dev);
    int ne = min(a.n_edge, n_rows);
    if (a.n_edge_dev) ne = min(ne, *a.n_edge_dev);
    n_rows = __builtin_amdgcn_readfirstlane(n_rows);
    const int n_tiles = __builtin_amdgcn_readfirstlane((max(ne, 0) + F2_ROWS - 1) / F2_ROWS);
    const int eW = a.exps[1];
    __builtin_amdgcn_s_waitcnt(0);  // (this wave's image DMAs landed)
    __syncthreads();
    const float *xb = a.x_dev ? gload(a.x_dev, 0) : a.x;
    const int32_t *colg = a.col_x ? a.col_x : a.col;  // the gather's source rows
    const int64_t xrows = a.col_x ? a.x_rows : static_cast<int64_t>(n_rows);
    const int64_t xbytes = (xrows - 1) * a.ldx * 4 + a.K0 * 4;
    const i32x4 xr = make_rsrc_u(xb, static_cast<uint32_t>(xrows > 0 ? xbytes : 0));
    const i32x4 ar = make_rsrc(a.agg, static_cast<uint32_t>(a.cap_rows * a.ld_agg * 4));
    const i32x4 nr = make_rsrc(a.nb, static_cast<uint32_t>(a.cap_rows * F2_HID * 4));
    const uint32_t ld4 = static_cast<uint32_t>(a.ldx) * 4u;
    const int q = ln >> 4, rl = ln & 15;
    for (int t = static_cast<int>(blockIdx.x) * F2_WAVES + wv; t < n_tiles; t += gridDim.x * F2_WAVES) {
        const int r = t * F2_ROWS + rl;
        const int beg = r < n_rows ? a.rowptr[r] : 0;
        const int deg = r < n_rows ? a.rowptr[r + 1] - beg : 0;
        // (the 16 rows' max degree: every row group holds the same 16 values)
        const int maxdeg = __builtin_amdgcn_readfirstlane(__float_as_int(max_row16(__int_as_float(deg))));
        // column offsets of the lane's 2 C0 pieces (past K0: out of range)
        int coff[2 * C0];
#pragma unroll
        for (int p = 0; p < 2 * C0; ++p) {
            const int k = 32 * (p >> 1) + 8 * q + 4 * (p & 1);
            coff[p] = k < a.K0 ? 4 * k : -1;
        }
        v4f acc[2 * C0];
#pragma unroll
        for (int p = 0; p < 2 * C0; ++p) acc[p] = v4f{0.f, 0.f, 0.f, 0.f};
        for (int e0 = 0; e0 < maxdeg; e0 += 16) {
            // the window's 16 neighbour ids first (one round trip), then the
            // rows, F2_NB per round trip
            int cw[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) cw[j] = e0 + j < deg ? gload(colg, beg + e0 + j) : -1;
#pragma unroll
            for (int b4 = 0; b4 < 16; b4 += F2_NB) {
                if (e0 + b4 >= maxdeg) break;
                v4f v[F2_NB][2 * C0];
#pragma unroll
                for (int u = 0; u < F2_NB; ++u) {
                    const int idx = cw[b4 + u];
                    const uint32_t ro = static_cast<uint32_t>(idx) * ld4;
#pragma unroll
                    for (int p = 0; p < 2 * C0; ++p)
                        v[u][p] = buf_load4(xr, (idx >= 0 && coff[p] >= 0) ? static_cast<int>(ro + coff[p]) : kOOB2,
                                            0, 0);
                }
#pragma unroll
                for (int u = 0; u < F2_NB; ++u)
#pragma unroll
                    for (int p = 0; p < 2 * C0; ++p) acc[p] += v[u][p];
            }
        }
        const float dv = static_cast<float>(deg > 1 ? deg : 1);
        float amax = 0.0f;
#pragma unroll
        for (int p = 0; p < 2 * C0; ++p) {
            if (a.mean) {
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[p][i] = acc[p][i] / dv;
            }
            amax = fmaxf(amax, amax4(acc[p]));
        }
        // the saved aggregate (rows of the edge tiles, columns < K0)
        const int arow = r < n_rows ? r * static_cast<int>(a.ld_agg) * 4 : kOOB2;
#pragma unroll
        for (int p = 0; p < 2 * C0; ++p)
            buf_store4(acc[p], ar, (coff[p] >= 0 && arow != kOOB2) ? arow + coff[p] : kOOB2, 0, 0);
        amax = max_xor32(max_xor16(amax));
        const int ea = h2_exp(amax);
        half8 b1[C0], b2[C0];
#pragma unroll
        for (int c = 0; c < C0; ++c) h2_split(ldexp4(acc[2 * c], ea), ldexp4(acc[2 * c + 1], ea), b1[c], b2[c]);
        const int un = -(eW + ea);
        const int nrow = r < n_rows ? r * F2_HID * 4 + 16 * q : kOOB2;
#pragma unroll 4
        for (int mt = 0; mt < F2_HID / 16; ++mt) {
            v4f o{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < C0; ++c) {
                const half8 w1 = simg[((mt * C0 + c) * 2) * 64 + ln];
                const half8 w2 = simg[((mt * C0 + c) * 2 + 1) * 64 + ln];
                o = mfma_h2(w1, w2, b1[c], b2[c], o);
            }
            buf_store4(ldexp4(o, un), nr, nrow == kOOB2 ? kOOB2 : nrow + 64 * mt, 0, 0);
        }
    }
}

// ---------------------------------------------------------------- k_fwd2
struct F2Args {
    const float *x;
    const float *const *x_dev;
    int64_t ldx;
    int K0;
    // fused x[n_id] gather: row r of the block is row xrow[r] of x (the
    // feature table, x_rows rows); the device word xrow_dev (graph slot, 0:
    // plain rows) overrides xrow; both null: identity
    const int64_t *xrow;
    const int64_t *const *xrow_dev;
    int64_t x_rows;
    int n_rows;
    const int32_t *n_rows_dev;
    int n_edge;
    const int32_t *n_edge_dev;
    const float *nb;  // [rows of the edge tiles, 256] (k_edge_nb)
    int64_t cap_rows;
    const half8 *img_r0, *img_1;
    const int *exps;
    const float *b0, *b1;
    Dropout drop;
    const uint64_t *seed_dev;
    float *h;  // [n, ldh]: rows < min(h_rows, *h_rows_dev) written
    int64_t ldh;
    int h_rows;
    const int32_t *h_rows_dev;
    float *out;  // [n, ldo]: b1 + h W_r1^T
    int64_t ldo;
    float *z;  // [n, ldz]: h W_l1^T
    int64_t ldz;
    int F1;
};

// DM: dropout mode (0 none, 1 byte, 2 bit: Dropout in ngnn_device.h).  XR:
// the fused x[n_id] gather (rows through n_id, whose loads run two tiles
// ahead of the row loads: a dependent index load next to them made every
// tile wait vmcnt(0) -- a drain of the prefetches and the previous stores)
template <int C0, int NT1, int DM, bool XR>
__global__ __launch_bounds__(F2_WAVES * 64) void k_fwd2(F2Args a) {
    constexpr int MT1 = 2 * NT1;
    constexpr int PSTR = 32 * C0 + 8;        // halves per row of a parts buffer (+16 B pad)
    constexpr int XPB = 2 * F2_ROWS * PSTR;  // halves per x-parts buffer (2 parts)
    constexpr int NIT = MT1 * 8;             // reduce items per wave (MT1 x 64 over 8 waves)
    extern __shared__ __attribute__((aligned(16))) v4f lds2[];
    v4f *spart = lds2;                                                   // [2][8][MT1][64]
    _Float16 *sxp = reinterpret_cast<_Float16 *>(lds2 + 2 * F2_WAVES * MT1 * 64);  // [2][2][16][PSTR]
    int *serow = reinterpret_cast<int *>(sxp + 2 * XPB);                // [2][16]

    const int wv = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int ln = threadIdx.x & 63, q = ln >> 4, rl = ln & 15;
    // ---- this wave's weight slices, for the whole launch
    half8 wr[2][C0][2], w1[MT1][2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int c = 0; c < C0; ++c)
#pragma unroll
            for (int p = 0; p < 2; ++p) wr[mt][c][p] = a.img_r0[((((wv * 2 + mt) * C0 + c) * 2) + p) * 64 + ln];
#pragma unroll
    for (int m = 0; m < MT1; ++m)
#pragma unroll
        for (int p = 0; p < 2; ++p) w1[m][p] = a.img_1[((wv * MT1 + m) * 2 + p) * 64 + ln];
    const int eW0 = __builtin_amdgcn_readfirstlane(a.exps[0]);
    const int eW1 = __builtin_amdgcn_readfirstlane(a.exps[2]);
    v4f b0v[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) b0v[mt] = *reinterpret_cast<const v4f *>(a.b0 + 32 * wv + 16 * mt + 4 * q);
    // reduce item of this lane (lanes < NIT): output tile mt1, lane lnn of it;
    // items [0, 64 NT1) are out's tiles, the rest z's -- waves 0-3 take out,
    // waves 4-7 z (NIT = 16 NT1 items per wave), so the store form is
    // wave-uniform (no exec-divergent store branches: their varying VMEM
    // counts made the compiler's waits conservative)
    const int item = wv * NIT + (ln < NIT ? ln : 0);
    const int rmt = item >> 6, rln = item & 63;
    const int rzt = __builtin_amdgcn_readfirstlane(wv) >= F2_WAVES / 2;
    const int rcol = 16 * (rmt - rzt * NT1) + 4 * (rln >> 4);  // first output column of the item
    v4f b1v{0.f, 0.f, 0.f, 0.f};
    if (!rzt) {
#pragma unroll
        for (int i = 0; i < 4; ++i) b1v[i] = rcol + i < a.F1 ? a.b1[rcol + i] : 0.0f;
    }
    Dropout drop = a.drop;
    if (a.seed_dev) drop.reseed(*a.seed_dev);

    int n_rows = a.n_rows;
    if (a.n_rows_dev) n_rows = min(n_rows, *a.n_rows_dev);
    int ne = min(a.n_edge, n_rows);
    if (a.n_edge_dev) ne = min(ne, *a.n_edge_dev);
    int hr = min(a.h_rows, n_rows);
    if (a.h_rows_dev) hr = min(hr, *a.h_rows_dev);
    n_rows = __builtin_amdgcn_readfirstlane(n_rows);
    ne = __builtin_amdgcn_readfirstlane(max(ne, 0));
    hr = __builtin_amdgcn_readfirstlane(max(hr, 0));
    const int n_tiles = (n_rows + F2_ROWS - 1) / F2_ROWS;
    const int G = gridDim.x, b = blockIdx.x;
    const int ntj = n_tiles > b ? (n_tiles - 1 - b) / G + 1 : 0;  // this workgroup's tiles
    if (ntj == 0) return;  // (uniform over the workgroup)

    const float *xb = a.x_dev ? gload(a.x_dev, 0) : a.x;
    const int64_t *xrow = !XR ? nullptr : a.xrow_dev ? gload(a.xrow_dev, 0) : a.xrow;
    const int64_t xrows = xrow ? a.x_rows : static_cast<int64_t>(n_rows);
    // (XR: n_id through a buffer resource -- a word of 0 means plain rows)
    const i32x4 ir = make_rsrc_u(xrow, static_cast<uint32_t>(xrow ? static_cast<int64_t>(n_rows) * 8 : 0));
    const int64_t xbytes = (xrows - 1) * a.ldx * 4 + a.K0 * 4;
    const i32x4 xr = make_rsrc_u(xb, static_cast<uint32_t>(xrows > 0 ? xbytes : 0));
    const int ne16 = (ne + F2_ROWS - 1) / F2_ROWS * F2_ROWS;
    const i32x4 nbr = make_rsrc(a.nb, static_cast<uint32_t>(static_cast<int64_t>(min<int64_t>(ne16, a.cap_rows)) * F2_HID * 4));
    const i32x4 hrs = make_rsrc(a.h, static_cast<uint32_t>(static_cast<int64_t>(hr) * a.ldh * 4));
    const i32x4 ors = make_rsrc(a.out, static_cast<uint32_t>(static_cast<int64_t>(n_rows) * a.ldo * 4));
    const i32x4 zrs = make_rsrc(a.z, static_cast<uint32_t>(static_cast<int64_t>(n_rows) * a.ldz * 4));
    const uint32_t ld4 = static_cast<uint32_t>(a.ldx) * 4u;

    // ---- x split lanes: row srow of the tile, columns 4 sslot .. + 3
    const int srow = 2 * wv + (ln >> 5), sslot = ln & 31;
    const bool scol = 4 * sslot < a.K0 && sslot < 8 * C0;
    auto tile_of = [&](int j) { return b + j * G; };
    // XR: the split row's feature-table index (low word of n_id; rows past
    // the block read 0 and are masked at use)
    auto iload = [&](int j) __attribute__((always_inline)) -> int {
        const int row = tile_of(j) * F2_ROWS + srow;
        return buf_load1i(ir, row < n_rows ? row * 8 : kOOB2, 0, 0);
    };
    auto xload = [&](int j, int idx) __attribute__((always_inline)) -> v4f {
        const int row = tile_of(j) * F2_ROWS + srow;
        const bool ok = j < ntj && row < n_rows && scol;
        const uint32_t src = (XR && xrow) ? static_cast<uint32_t>(idx) : static_cast<uint32_t>(row);
        return buf_load4(xr, ok ? static_cast<int>(src * ld4 + 16u * sslot) : kOOB2, 0, 0);
    };
    // nb of the lane's 8 columns (rows past the edge tiles read 0)
    auto nbload = [&](int j, v4f (&nbv)[2]) __attribute__((always_inline)) {
        const int row = tile_of(j) * F2_ROWS + rl;
        const bool ok = j < ntj && row < ne16;
        const int o = ok ? row * F2_HID * 4 + (32 * wv + 4 * q) * 4 : kOOB2;
        nbv[0] = buf_load4(nbr, o, 0, 0);
        nbv[1] = buf_load4(nbr, o == kOOB2 ? kOOB2 : o + 64, 0, 0);
    };
    // row max over the tile row's 32 lanes, scale, split, parts into LDS
    auto split = [&](v4f v, int buf) __attribute__((always_inline)) {
        const float m = max_xor16(max_row16(amax4(v)));  // the tile row's 32 lanes
        const int e = h2_exp(m);
        const v4f vs = ldexp4(v, e);
        half4 p1, p2;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const _Float16 hh = static_cast<_Float16>(vs[i]);
            p1[i] = hh;
            p2[i] = static_cast<_Float16>(vs[i] - static_cast<float>(hh));
        }
        if (sslot < 8 * C0) {
            _Float16 *d = sxp + buf * XPB + srow * PSTR + 4 * sslot;
            *reinterpret_cast<half4 *>(d) = p1;
            *reinterpret_cast<half4 *>(d + F2_ROWS * PSTR) = p2;
        }
        if (sslot == 0) serow[buf * F2_ROWS + srow] = e;
    };
    // one tile: layer 0 (32 columns), epilogue, h rows, layer-1 partial
    auto compute = [&](int j, int buf, const v4f (&nbv)[2]) __attribute__((always_inline)) {
        const int t = tile_of(j);
        const int r = t * F2_ROWS + rl;
        v4f acc[2] = {v4f{0.f, 0.f, 0.f, 0.f}, v4f{0.f, 0.f, 0.f, 0.f}};
        const _Float16 *xp = sxp + buf * XPB + rl * PSTR + 8 * q;
#pragma unroll
        for (int c = 0; c < C0; ++c) {
            const half8 x1 = *reinterpret_cast<const half8 *>(xp + 32 * c);
            const half8 x2 = *reinterpret_cast<const half8 *>(xp + F2_ROWS * PSTR + 32 * c);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) acc[mt] = mfma_h2(wr[mt][c][0], wr[mt][c][1], x1, x2, acc[mt]);
        }
        const int un0 = -(eW0 + serow[buf * F2_ROWS + rl]);
        // epilogue: b0 + x W_r0^T + nb, ReLU (NaN passes), dropout keyed by
        // (global row, global column) exactly as every other forward kernel
        const uint32_t rk = DM ? drop.row_key(static_cast<uint32_t>(r)) : 0u;
        const uint32_t hw = DM == 2 ? lowbias32(rk + static_cast<uint32_t>(wv)) : 0u;  // columns 32 wv .. + 31
        v4f hv[2];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            const uint32_t hq = DM == 1 ? lowbias32(rk + static_cast<uint32_t>(8 * wv + 4 * mt + q)) : 0u;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float y = __builtin_amdgcn_ldexpf(acc[mt][i], un0) + b0v[mt][i] + nbv[mt][i];
                bool zero = y < 0.0f;
                if (DM == 2) zero = zero || !((hw >> (16 * mt + 4 * q + i)) & 1u);
                if (DM == 1) zero = zero || ((hq >> (8 * i)) & 0xffu) < drop.thresh;
                hv[mt][i] = zero ? 0.0f : (DM ? y * drop.scale : y);
            }
        }
        // h rows the backward reads (past the bound: dropped by the range)
        const int ho = static_cast<int>(static_cast<uint32_t>(r) * static_cast<uint32_t>(a.ldh) * 4u) + (32 * wv + 4 * q) * 4;
        buf_store4(hv[0], hrs, r < hr ? ho : kOOB2, 0, 0);
        buf_store4(hv[1], hrs, r < hr ? ho + 64 : kOOB2, 0, 0);
        // layer 1: this wave's 32 rows of K -- the B fragment is the lane's own
        // 8 values of h (k order 4q + i, 16 + 4q + i: the image matches)
        const float m = max_xor32(max_xor16(fmaxf(amax4(hv[0]), amax4(hv[1]))));  // lanes rl + 16 q
        const int eh = h2_exp(m);
        half8 h1, h2;
        h2_split(ldexp4(hv[0], eh), ldexp4(hv[1], eh), h1, h2);
        const int un1 = -(eW1 + eh);
        v4f *pp = spart + (buf * F2_WAVES + wv) * MT1 * 64 + ln;
#pragma unroll
        for (int m1 = 0; m1 < MT1; ++m1) {
            const v4f o = mfma_h2(w1[m1][0], w1[m1][1], h1, h2, v4f{0.f, 0.f, 0.f, 0.f});
            pp[m1 * 64] = ldexp4(o, un1);
        }
    };
    // the 8 partials of this lane's item, summed in wave order (+ b1), stored
    auto reduce = [&](int j, int buf) __attribute__((always_inline)) {
        const v4f *pp = spart + buf * F2_WAVES * MT1 * 64 + rmt * 64 + rln;
        v4f s = pp[0];
#pragma unroll
        for (int w = 1; w < F2_WAVES; ++w) s += pp[w * MT1 * 64];
        const int row = tile_of(j) * F2_ROWS + (rln & 15);
        const bool live = ln < NIT && row < n_rows;
        if (rzt) {
            const int zo = live ? static_cast<int>(static_cast<uint32_t>(row) * static_cast<uint32_t>(a.ldz) * 4u) + 4 * rcol : kOOB2;
            buf_store4(s, zrs, zo, 0, 0);
        } else {
            s += b1v;
            const int oo = static_cast<int>(static_cast<uint32_t>(row) * static_cast<uint32_t>(a.ldo) * 4u) + 4 * rcol;
#pragma unroll
            for (int i = 0; i < 4; ++i) buf_store1(s[i], ors, (live && rcol + i < a.F1) ? oo + 4 * i : kOOB2, 0, 0);
        }
    };

    // ---- pipeline: x of 4 tiles in flight (registers, one buffer per tile
    // residue mod 4); per tile j: split(j + 1), compute(j), ONE barrier,
    // reduce(j).  Double-buffered parts and partials make the single barrier
    // sufficient.
    //
    // vmcnt counts vector-memory ops IN ORDER, so a load consumed soon after
    // its issue forces every older one -- the x prefetches -- to land with
    // it.  Hence: (1) the edge tiles (nb, loaded one tile ahead) run in a
    // phase of their own (the first ~4 tiles of a workgroup), the other tiles
    // in a phase without nb loads; (2) XR's n_id loads run four tiles ahead
    // of the row loads that use them; (3) loads pending at a phase entry are
    // SETTLED first -- the compiler's wait for a loop-carried load takes the
    // fewest younger memory ops over the paths into the loop, and a load left
    // pending on the entry path made every in-loop wait a near drain of the
    // prefetches and the previous tiles' stores (vmcnt(4) instead of ~20).
    v4f xv[4];
    int ixr[4] = {0, 0, 0, 0};  // XR: n_id of tile j + 5 at step j (slot j % 4)
#pragma unroll
    for (int i = 0; i < 4; ++i) xv[i] = xload(i, XR ? iload(i) : 0);
    v4f nbv[2][2];
    nbload(0, nbv[0]);
    split(xv[0], 0);
    xv[0] = xload(4, XR ? iload(4) : 0);
    if (XR) {
#pragma unroll
        for (int i = 0; i < 4; ++i) ixr[i] = iload(5 + i);
    }
    auto settle = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(xv[i]), "+v"(ixr[i]));
        asm volatile("" : "+v"(nbv[0][0]), "+v"(nbv[0][1]), "+v"(nbv[1][0]), "+v"(nbv[1][1]));
    };
    settle();
    lds_barrier();
    auto step = [&](auto u_c, auto nb_c, int j) __attribute__((always_inline)) {
        constexpr int U = decltype(u_c)::value;   // j % 4
        constexpr int B = U & 1;                  // j % 2
        constexpr bool NB = decltype(nb_c)::value;  // an edge tile phase
        // (unconditional: past the last tile it splits zeros into a parts
        // buffer no one reads -- a skipped split left that register's load
        // pending on one path, and the compiler then drained vmcnt before
        // reusing the register)
        split(xv[(U + 1) & 3], B ^ 1);
        xv[(U + 1) & 3] = xload(j + 5, ixr[U]);
        if (XR) ixr[U] = iload(j + 9);
        if (NB) {
            nbload(j + 1, nbv[B ^ 1]);
            compute(j, B, nbv[B]);
        } else {
            const v4f zz[2] = {v4f{0.f, 0.f, 0.f, 0.f}, v4f{0.f, 0.f, 0.f, 0.f}};
            compute(j, B, zz);
        }
        lds_barrier();
        reduce(j, B);
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    // this workgroup's edge tiles: j < ntj_e, rounded up to a multiple of 4
    // (the ring position); tiles past the edge rows in it read nb = 0
    const int n_et = ne16 / F2_ROWS;
    const int ntj_e = min(ntj, 4 * ((max(0, (n_et - b + G - 1) / G) + 3) / 4));
    int j = 0;
    for (; j < ntj_e; j += 4) {
        step(I0{}, std::true_type{}, j);
        if (j + 1 >= ntj) break;
        step(I1{}, std::true_type{}, j + 1);
        if (j + 2 >= ntj) break;
        step(I2{}, std::true_type{}, j + 2);
        if (j + 3 >= ntj) break;
        step(I3{}, std::true_type{}, j + 3);
    }
    if (j >= ntj) return;
    settle();  // (the x rows in flight: settled once at the phase change)
    // whole trips of 4 steps with no exits inside (an exit between steps
    // gave the compiler's wait analysis a short path into the loop head:
    // vmcnt(2) there, a near drain every 4 tiles), then the remainder
    for (; j + 4 <= ntj; j += 4) {
        step(I0{}, std::false_type{}, j);
        step(I1{}, std::false_type{}, j + 1);
        step(I2{}, std::false_type{}, j + 2);
        step(I3{}, std::false_type{}, j + 3);
    }
    if (j < ntj) step(I0{}, std::false_type{}, j);
    if (j + 1 < ntj) step(I1{}, std::false_type{}, j + 1);
    if (j + 2 < ntj) step(I2{}, std::false_type{}, j + 2);
}

template <int C0, int NT1, int DM, bool XR>
int launch_fwd2(const F2Args &a, int grid, hipStream_t st) {
    auto fn = k_fwd2<C0, NT1, DM, XR>;
    const size_t lds = static_cast<size_t>(2) * F2_WAVES * 2 * NT1 * 64 * 16 +
                       static_cast<size_t>(2) * 2 * F2_ROWS * (32 * C0 + 8) * 2 + 2 * F2_ROWS * 4;
    static bool attr_set = false;  // benign race: idempotent
    if (!attr_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(F2_WAVES * 64), lds, st, a);
    return launch_status();
}

template <int C0>
int launch_edge_nb(const G2Args &a, int grid, hipStream_t st) {
    auto fn = k_edge_nb<C0>;
    const size_t lds = static_cast<size_t>(F2_HID / 16) * C0 * 2 * 64 * 16;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(F2_WAVES * 64), lds, st, a);
    return launch_status();
}

// workspace layout (16-B aligned pieces)
struct Ws2 {
    size_t img_r0, img_l0, img_1, exps, nb, z, total;
};
Ws2 ws2_layout(int64_t K0, int64_t F1, int64_t n_rows) {
    const int64_t C0 = ceil_div(K0, 32), NT1 = ceil_div(F1, 16);
    Ws2 w;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += (bytes + 255) & ~size_t(255);
        return o;
    };
    w.img_r0 = take(static_cast<size_t>(F2_WAVES) * 2 * C0 * 2 * 64 * 16);
    w.img_l0 = take(static_cast<size_t>(F2_HID / 16) * C0 * 2 * 64 * 16);
    w.img_1 = take(static_cast<size_t>(F2_WAVES) * 2 * NT1 * 2 * 64 * 16);
    w.exps = take(16);
    const int64_t rows16 = ceil_div(std::max<int64_t>(n_rows, 1), 16) * 16;
    w.nb = take(static_cast<size_t>(rows16) * F2_HID * 4);
    w.z = take(static_cast<size_t>(rows16) * NT1 * 16 * 4);
    w.total = off;
    return w;
}

}  // namespace

// narrow-mode neighbour term (ngnn_sage_rt.hip)
int narrow_agg_launch(const float *z, int64_t ldz, int64_t Fo, const int32_t *rowptr, const int32_t *col,
                      int64_t n_rows, const int32_t *n_rows_dev, int64_t n_edge_rows,
                      const int32_t *n_edge_rows_dev, int reduce, float *out, int64_t ldo, hipStream_t st);

}  // namespace ngnn

using namespace ngnn;

extern "C" int ngnn_sage2_supported(int64_t K0, int64_t H, int64_t F1, int reduce) {
    return (K0 > 96 && K0 <= 128 && K0 % 4 == 0 && H == F2_HID && F1 > 32 && F1 <= 48 &&
            (reduce == NGNN_REDUCE_MEAN || reduce == NGNN_REDUCE_SUM))
               ? 1
               : 0;
}

extern "C" size_t ngnn_sage2_workspace_bytes(int64_t K0, int64_t F1, int64_t n_rows) {
    return ws2_layout(K0, F1, n_rows).total + 256;
}

extern "C" int ngnn_sage2_fwd(const float *x, const float *const *x_dev, const int64_t *xrow,
                              const int64_t *const *xrow_dev, int64_t x_rows, int64_t ldx, int64_t K0,
                              int64_t n_rows, const int32_t *n_rows_dev, int64_t n_edge_rows,
                              const int32_t *n_edge_rows_dev, const int32_t *rowptr, const int32_t *col,
                              const int32_t *col_x, int reduce, const float *wl0, const float *bl0, const float *wr0,
                              int64_t ldw0, int64_t H, const float *wl1, const float *bl1,
                              const float *wr1, int64_t ldw1, int64_t F1, float p_drop, uint64_t seed,
                              const uint64_t *seed_dev, float *h, int64_t ldh, int64_t h_rows,
                              const int32_t *h_rows_dev, float *agg0, int64_t ld_agg, float *out,
                              int64_t ldo, int stages, void *ws, size_t ws_bytes, void *stream) {
    NGNN_RETURN_IF(!ngnn_sage2_supported(K0, H, F1, reduce), NGNN_E_SHAPE);
    NGNN_RETURN_IF(n_rows < 0 || n_edge_rows < 0 || h_rows < 0, NGNN_E_ARG);
    NGNN_RETURN_IF(p_drop < 0.0f || !(p_drop <= 1.0f), NGNN_E_ARG);
    NGNN_RETURN_IF(stages <= 0 || stages > NGNN_SAGE2_ALL, NGNN_E_ARG);
    NGNN_RETURN_IF(ldx < K0 || ldx % 4 != 0 || ldw0 < K0 || ldw0 % 4 != 0 || ldw1 < H || ldw1 % 4 != 0 || ldh < H || ldh % 4 != 0 ||
                       ld_agg < K0 || ld_agg % 4 != 0 || ldo < F1,
                   NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(n_rows), NGNN_E_RANGE);
    const bool indexed = xrow || xrow_dev;
    NGNN_RETURN_IF(indexed && (x_rows <= 0 || !col_x), NGNN_E_ARG);
    if (n_rows == 0) return NGNN_OK;
    NGNN_RETURN_IF((!x && !x_dev) || !rowptr || (!col && n_edge_rows > 0) || !wl0 || !bl0 || !wr0 || !wl1 || !bl1 || !wr1 ||
                       !h || !agg0 || !out || !ws,
                   NGNN_E_ARG);
    NGNN_RETURN_IF((x && !aligned(x, 16)) || !aligned(h, 16) || !aligned(agg0, 16) || !aligned(bl0, 16) ||
                       !aligned(wr0, 16) || !aligned(wl0, 16) || !aligned(wr1, 16) || !aligned(wl1, 16) ||
                       !aligned(ws, 256),
                   NGNN_E_ALIGN);
    // 32-bit buffer offsets: every operand under 3.75 GiB
    const int64_t lim = 0xF0000000ll - 4096;
    NGNN_RETURN_IF(std::max(n_rows, indexed ? x_rows : 0) * ldx * 4 > lim || n_rows * ldh * 4 > lim || n_rows * ld_agg * 4 > lim ||
                       n_rows * ldo * 4 > lim || n_rows * F2_HID * 4 > lim,
                   NGNN_E_RANGE);
    const Ws2 L = ws2_layout(K0, F1, n_rows);
    NGNN_RETURN_IF(ws_bytes < L.total, NGNN_E_WORKSPACE);
    hipStream_t st = as_stream(stream);
    char *wsb = static_cast<char *>(ws);
    const int C0 = static_cast<int>(ceil_div(K0, 32)), NT1 = static_cast<int>(ceil_div(F1, 16));
    half8 *img_r0 = reinterpret_cast<half8 *>(wsb + L.img_r0);
    half8 *img_l0 = reinterpret_cast<half8 *>(wsb + L.img_l0);
    half8 *img_1 = reinterpret_cast<half8 *>(wsb + L.img_1);
    int *exps = reinterpret_cast<int *>(wsb + L.exps);
    float *nb = reinterpret_cast<float *>(wsb + L.nb);
    float *z = reinterpret_cast<float *>(wsb + L.z);
    const int64_t ldz = 16 * NT1;
    const int64_t cap_rows = ceil_div(n_rows, 16) * 16;
    // the saved aggregate's and nb's rows: whole edge tiles (NB: agg0 must hold
    // ceil16(n_edge) rows when they exceed n_rows -- capped at n_rows here)
    if (stages & NGNN_SAGE2_PREP) {
        P2Args p{wr0, wl0, ldw0, static_cast<int>(K0), C0, wr1, wl1, ldw1, static_cast<int>(F1), NT1,
                 img_r0, img_l0, img_1, exps};
        // (F2_WAVES * 2 * C0 * 64 = 4,096 slots of the largest image: 16 blocks each)
        hipLaunchKernelGGL(k_prep2, dim3(16, 3), dim3(P2_THREADS), 0, st, p);
        const int rc = launch_status();
        if (rc) return rc;
    }
    const int ncu = num_cus();
    if ((stages & NGNN_SAGE2_EDGE) && n_edge_rows > 0) {
        G2Args g;
        g.x = x;
        g.x_dev = x_dev;
        g.ldx = ldx;
        g.K0 = static_cast<int>(K0);
        g.n_rows = static_cast<int>(n_rows);
        g.n_rows_dev = n_rows_dev;
        g.n_edge = static_cast<int>(std::min(n_edge_rows, n_rows));
        g.n_edge_dev = n_edge_rows_dev;
        g.rowptr = rowptr;
        g.col = col;
        g.col_x = indexed ? col_x : nullptr;
        g.x_rows = x_rows;
        g.mean = reduce == NGNN_REDUCE_MEAN;
        g.img_l0 = img_l0;
        g.exps = exps;
        g.agg = agg0;
        g.ld_agg = ld_agg;
        g.nb = nb;
        g.cap_rows = n_rows;  // (agg0 has n_rows rows; nb has cap_rows >= n_rows)
        const int tiles = static_cast<int>(ceil_div(g.n_edge, 16));
        const int grid = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(ncu, ceil_div(tiles, F2_WAVES))));
        int rc = NGNN_E_SHAPE;
        if (C0 == 4) rc = launch_edge_nb<4>(g, grid, st);
        if (rc) return rc;
    }
    if (stages & NGNN_SAGE2_MAIN) {
        F2Args f;
        f.x = x;
        f.x_dev = x_dev;
        f.ldx = ldx;
        f.K0 = static_cast<int>(K0);
        f.xrow = xrow;
        f.xrow_dev = xrow_dev;
        f.x_rows = x_rows;
        f.n_rows = static_cast<int>(n_rows);
        f.n_rows_dev = n_rows_dev;
        f.n_edge = static_cast<int>(std::min(n_edge_rows, n_rows));
        f.n_edge_dev = n_edge_rows_dev;
        f.nb = nb;
        f.cap_rows = cap_rows;
        f.img_r0 = img_r0;
        f.img_1 = img_1;
        f.exps = exps;
        f.b0 = bl0;
        f.b1 = bl1;
        f.drop = make_dropout(p_drop, seed);
        f.seed_dev = seed_dev;
        f.h = h;
        f.ldh = ldh;
        f.h_rows = static_cast<int>(std::min(h_rows, n_rows));
        f.h_rows_dev = h_rows_dev;
        f.out = out;
        f.ldo = ldo;
        f.z = z;
        f.ldz = ldz;
        f.F1 = static_cast<int>(F1);
        const int64_t tiles = ceil_div(n_rows, 16);
        const int grid = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(ncu, tiles)));
        const int dm = f.drop.thresh == 0 ? 0 : f.drop.thresh == 128u ? 2 : 1;
        int rc = NGNN_E_SHAPE;
        auto go = [&](auto xr_c) {
            constexpr bool XRv = decltype(xr_c)::value;
            return dm == 2   ? launch_fwd2<4, 3, 2, XRv>(f, grid, st)
                   : dm == 1 ? launch_fwd2<4, 3, 1, XRv>(f, grid, st)
                             : launch_fwd2<4, 3, 0, XRv>(f, grid, st);
        };
        if (C0 == 4 && NT1 == 3) rc = indexed ? go(std::true_type{}) : go(std::false_type{});
        if (rc) return rc;
    }
    if (!(stages & NGNN_SAGE2_NARROW)) return NGNN_OK;
    return narrow_agg_launch(z, ldz, F1, rowptr, col, n_rows, n_rows_dev, n_edge_rows, n_edge_rows_dev, reduce,
                             out, ldo, st);
}
