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
// Two launches (plus the narrow neighbour term), all on the caller's stream;
// each loads its weight slices into registers itself (per-wave scales):
//   k_edge_nb  rows with in-edges (NeighborLoader numbers them first): the
//              neighbour aggregate in edge order (bit-identical to
//              ngnn_seg_agg_fwd; it is the backward's saved aggregate), then
//              nb = agg W_l0^T on MFMA, W_l0's slices in registers;
//   k_fwd2     every row: layer 0's root term + nb + epilogue, layer 1's
//              products, the cross-wave sum; then k_narrow_agg (ngnn_sage_rt.hip)
//              adds mean_j z_j to the rows with in-edges.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "ngnn_device.h"

namespace ngnn {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float v2f __attribute__((ext_vector_type(2)));

constexpr int F2_WAVES = 8;    // workgroup: 8 waves x 32 hidden columns = 256
constexpr int F2_HID = 256;    // hidden width of the fused shape
constexpr int F2_ROWS = 16;    // rows per tile (one MFMA n-block)
constexpr int kOOB2 = static_cast<int>(0xF0000000u);  // past every buffer range
#ifndef NGNN_F2_STAUX
#define NGNN_F2_STAUX 2  // the main phase's h / out / z stores non-temporal (nt): fused launch 93.7 -> 89.6 us (A/B, r06g)
#endif
// (per-output overrides: the consumers -- the narrow launch gathers z rows
// and updates out, k_bwd2 reads h rows < R' -- prefer those rows cached.  z
// cached: the narrow launch's z gather hits L2 / MALL, step span 168.0 ->
// 161.4 us; h cached on top: k_bwd2's h reads too, span 166.6 -> 158.8 us;
// out cached: no change (profiles/r06sa_store_policy_ab.txt,
// profiles/r06sb_store_policy_ab.txt))
#ifndef NGNN_F2_STAUX_H
#define NGNN_F2_STAUX_H 0
#endif
#ifndef NGNN_F2_STAUX_Z
#define NGNN_F2_STAUX_Z 0
#endif
#ifndef NGNN_F2_STAUX_O
#define NGNN_F2_STAUX_O NGNN_F2_STAUX
#endif

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

// ---------------------------------------------------------------- weight slices
// Every wave loads its slice of a weight matrix straight from the fp32
// weights into A-fragment registers at launch (~100 KB per matrix per
// workgroup, L2-resident after the first workgroups): lane (m, q) of a
// fragment holds 8 values of one weight row (two 16-B loads), scaled by the
// wave's OWN power of two (max |w| over the wave's slice) and split into the
// two fp16 parts.  Per-wave scales are exact to undo: every product is
// unscaled per wave before any cross-wave sum -- so there is no weight-prep
// launch and no cross-workgroup hand-off (a round-3 design had both).

// layer 0's slice of wave wv: rows 32 wv + 16 mt + m of w ([256, K0], row
// stride ldw), k = 32 c + 8 q .. + 7; returns the wave's exponent
// (in two halves, so a caller can issue other loads between the slice's
// loads and their use: w0_slice_issue, then w0_slice_finish)
// (buffer loads, as the callers' other loads: the compiler counts them in
// issue order with the rest -- mixed with global loads it waited for the
// whole slice before the first index word)
template <int C0>
__device__ __forceinline__ void w0_slice_issue(const float *w, int64_t ldw, int K0, int wv, int ln,
                                               v4f (&t)[2][C0][2]) {
    const int q = ln >> 4, m = ln & 15;
    const i32x4 wr = make_rsrc(w, static_cast<uint32_t>(static_cast<int64_t>(F2_HID) * ldw * 4));
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
        const int rb = (32 * wv + 16 * mt + m) * static_cast<int>(ldw) * 4;
#pragma unroll
        for (int c = 0; c < C0; ++c)
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                const int k = 32 * c + 8 * q + 4 * p;
                t[mt][c][p] = buf_load4(wr, k < K0 ? rb + 4 * k : kOOB2, 0, 0);
            }
    }
}
template <int C0>
__device__ __forceinline__ int w0_slice_finish(const v4f (&t)[2][C0][2], half8 (&frag)[2][C0][2]) {
    float mx = 0.0f;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int c = 0; c < C0; ++c)
#pragma unroll
            for (int p = 0; p < 2; ++p) mx = fmaxf(mx, amax4(t[mt][c][p]));
    const int e = __builtin_amdgcn_readfirstlane(h2_exp(wave_max(mx)));
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int c = 0; c < C0; ++c) h2_split(ldexp4(t[mt][c][0], e), ldexp4(t[mt][c][1], e), frag[mt][c][0], frag[mt][c][1]);
    return e;
}
template <int C0>
__device__ __forceinline__ int load_w0_slice(const float *w, int64_t ldw, int K0, int wv, int ln,
                                             half8 (&frag)[2][C0][2]) {
    v4f t[2][C0][2];
    w0_slice_issue<C0>(w, ldw, K0, wv, ln, t);
    return w0_slice_finish<C0>(t, frag);
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
    const float *wl0;  // [256, K0], row stride ldw0
    int64_t ldw0;
    float *agg;  // saved aggregate [>= rows of the edge tiles, ld_agg]
    int64_t ld_agg;
    float *nb;   // [>= rows of the edge tiles, 256]
    int64_t cap_rows;  // rows of agg / nb
    // the loss head's g (nullable): rows < min(gz_rows, *gz_rows_dev) of
    // gz_ld floats (a multiple of 4) are zeroed here, before its scatter
    float *gz;
    int gz_ld;
    int gz_rows;
    const int32_t *gz_rows_dev;
    // ... and its valid-label count: #{i < cnt_B : cnt_y[i] != cnt_ignore}
    // into *cnt_out (nullable), by the last workgroup
    const int64_t *cnt_y;
    int cnt_B;
    int64_t cnt_ignore;
    float *cnt_out;
    // ... and the head's seed-edge counts per source (nullable, NarrowHead's
    // scnt_*): counted into the selected array, the other one cleared
    int32_t *scnt_base;
    int scnt_stride;
};

constexpr int G2_NB = 16;  // neighbour rows in flight per lane (one round trip for fanouts <= 16)

// The rows with in-edges, 16-row tiles, one workgroup (8 waves) per CU
// walking its tiles.  Per tile: every wave gathers TWO rows (32 lanes x 4
// columns per row: the x split layout of k_fwd2), all of a row's neighbours
// in one round trip, sums them in edge order from +0.0 and divides by
// max(deg, 1) for mean -- the fp32 sequence of ngnn_seg_agg_fwd (the saved
// aggregate is bit-identical to it); stores the aggregate, splits it into
// fp16 parts in LDS; after one barrier every wave multiplies the tile by ITS
// 32 columns of W_l0 (slice in registers) and stores nb, unscaled.
//
// Two tiles' gathers in flight: the rows of tile j+1 are requested BEFORE
// tile j is consumed (they land during its sum, split, barrier and MFMAs),
// the neighbour ids two tiles ahead, the row pointers three.  vmcnt retires
// in issue order, so every index word a request needs was issued before the
// rows still in flight (per step: rowptr(j+3), ids(j+2), rows(j+1), then
// tile j) and waiting on it never drains them.  A row's ids are spread over
// its 32 lanes (lane s holds neighbour s: one word per lane per tile) and
// broadcast with bpermute at the request.  The first tile's rows are
// requested before the weight slices load (the two latencies overlap).
// DBG (profiling builds only, NGNN_EDGE_DBG): bit 0 skips the row gathers
// (out-of-range requests), 1 the MFMAs and nb stores, 2 the aggregate stores
// (the body, shared by k_edge_nb and the fused k_fwd2x below)
template <int C0, int DBG = 0>
__device__ __forceinline__ void edge_nb_body(const G2Args &a) {
    constexpr int PSTR = 32 * C0 + 16;  // 72 dwords = 8 mod 64 banks: conflict-free fragment reads
    constexpr int XPB = 2 * F2_ROWS * PSTR;
    __shared__ __attribute__((aligned(16))) _Float16 sxp[2 * XPB];
    __shared__ int serow[2 * F2_ROWS];
    __shared__ __attribute__((aligned(16))) int sid[64 * F2_WAVES];
    const int wv = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int ln = threadIdx.x & 63, q = ln >> 4, rl = ln & 15;
    int n_rows = a.n_rows;
    if (a.n_rows_dev) n_rows = min(n_rows, *a.n_rows_dev);
    int ne = min(a.n_edge, n_rows);
    if (a.n_edge_dev) ne = min(ne, *a.n_edge_dev);
    n_rows = __builtin_amdgcn_readfirstlane(n_rows);
    const int n_tiles = __builtin_amdgcn_readfirstlane((max(ne, 0) + F2_ROWS - 1) / F2_ROWS);
    const int G = gridDim.x, b = blockIdx.x;
    if (a.gz) {  // the loss head's g rows, spread over the whole grid
        int gr = a.gz_rows;
        if (a.gz_rows_dev) gr = min(gr, *a.gz_rows_dev);
        gr = max(gr, 0);
        const int n4 = gr * (a.gz_ld >> 2);
        for (int i = b * (F2_WAVES * 64) + static_cast<int>(threadIdx.x); i < n4; i += G * F2_WAVES * 64)
            reinterpret_cast<v4f *>(a.gz)[i] = v4f{0.f, 0.f, 0.f, 0.f};
        if (a.scnt_base) {
            // this call's counts: one per edge into a seed row, by source (the
            // array the head reads); the other array -- read by the previous
            // call's head -- back to zero for the next call (rows < R': the
            // sources any seed edge had; rows past it only ever over-count)
            const int sel = a.scnt_base[2 * a.scnt_stride] & 1;
            int32_t *cn = a.scnt_base + sel * a.scnt_stride;
            int32_t *co = a.scnt_base + (sel ^ 1) * a.scnt_stride;
            const int nc = min(gr, a.scnt_stride);
            for (int i = b * (F2_WAVES * 64) + static_cast<int>(threadIdx.x); i < nc; i += G * F2_WAVES * 64) co[i] = 0;
            const int es = a.rowptr[min(a.cnt_B, n_rows)];
            for (int e = b * (F2_WAVES * 64) + static_cast<int>(threadIdx.x); e < es; e += G * F2_WAVES * 64) {
                const int s = a.col[e];
                if (static_cast<unsigned>(s) < static_cast<unsigned>(a.scnt_stride)) atomicAdd(cn + s, 1);
            }
        }
    }
    if (a.cnt_out && b == G - 1) {  // (the last workgroup: the fewest tiles)
        __shared__ float s_cnt[F2_WAVES];
        float c = 0.0f;
        for (int i = threadIdx.x; i < a.cnt_B; i += F2_WAVES * 64) c += (a.cnt_y[i] != a.cnt_ignore) ? 1.0f : 0.0f;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
        if (ln == 0) s_cnt[wv] = c;
        __syncthreads();
        if (threadIdx.x == 0) {
            float t = 0.0f;
            for (int w = 0; w < F2_WAVES; ++w) t += s_cnt[w];
            *a.cnt_out = t;
        }
    }
    const int ntj = n_tiles > b ? (n_tiles - 1 - b) / G + 1 : 0;
    if (ntj == 0) return;  // (uniform over the workgroup)

    const float *xb = a.x_dev ? gload(a.x_dev, 0) : a.x;
    const int32_t *colg = a.col_x ? a.col_x : a.col;  // the gather's source rows
    const int64_t xrows = a.col_x ? a.x_rows : static_cast<int64_t>(n_rows);
    const int64_t xbytes = (xrows - 1) * a.ldx * 4 + a.K0 * 4;
    const i32x4 xr = make_rsrc_u(xb, static_cast<uint32_t>(xrows > 0 ? xbytes : 0));
    const i32x4 ar = make_rsrc(a.agg, static_cast<uint32_t>(a.cap_rows * a.ld_agg * 4));
    const i32x4 nr = make_rsrc(a.nb, static_cast<uint32_t>(a.cap_rows * F2_HID * 4));
    const uint32_t ld4 = static_cast<uint32_t>(a.ldx) * 4u;
    // gather lanes: row srow of the tile, columns 4 sslot .. + 3
    const int srow = 2 * wv + (ln >> 5), sslot = ln & 31;
    const bool scol = 4 * sslot < a.K0 && sslot < 8 * C0;
    auto tile_row = [&](int j, int rr) { return (b + j * G) * F2_ROWS + rr; };
    // index words through buffer resources (no branches, 32-bit offsets;
    // out-of-range slots read 0 and are masked by the degree at use; a tile
    // past the last reads beg = end = 0: no rows)
    const i32x4 rpr = make_rsrc(a.rowptr, static_cast<uint32_t>(static_cast<int64_t>(n_rows + 1) * 4));
    const i32x4 cr = make_rsrc(colg, 0xF0000000u);
    auto rowptr_of = [&](int j, int &beg, int &end) __attribute__((always_inline)) {
        const int r = tile_row(j, srow);
        const bool ok = j < ntj && r < n_rows;
        beg = buf_load1i(rpr, ok ? 4 * r : kOOB2, 0, 0);
        end = buf_load1i(rpr, ok ? 4 * r + 4 : kOOB2, 0, 0);
    };
    // lane sslot of the row's 32 holds neighbour e0 + sslot's id
    auto ids_of = [&](int beg, int end, int e0) __attribute__((always_inline)) {
        return buf_load1i(cr, beg + e0 + sslot < end ? 4 * (beg + e0 + sslot) : kOOB2, 0, 0);
    };
    // (row offsets as 24-bit products: every row of a table under the 32-bit
    // offset limit has an index < 2^24, and ld4 < 2^24)
    // (the row's ids pass through LDS: one word written per lane, the 16 in
    // use read back as four broadcast 16-B reads -- a wave's own LDS accesses
    // stay in order, no barrier)
    int *const sidr = sid + 64 * wv + (ln & 32);
    auto rows_of = [&](int beg, int end, int e0, int idl, v4f (&v)[G2_NB]) __attribute__((always_inline)) {
        sidr[sslot] = idl;
        int id[G2_NB];
#pragma unroll
        for (int k = 0; k < G2_NB / 4; ++k) {
            const i32x4 w = *reinterpret_cast<const i32x4 *>(sidr + ((e0 & 31) + 4 * k));
#pragma unroll
            for (int i = 0; i < 4; ++i) id[4 * k + i] = w[i];
        }
#pragma unroll
        for (int e = 0; e < G2_NB; ++e)
            v[e] = buf_load4(xr, (beg + e0 + e < end && scol && !(DBG & 1)) ? static_cast<int>(__umul24(static_cast<uint32_t>(id[e]), ld4) + 16u * sslot) : kOOB2,
                             0, 0);
    };

    // tile j (its rows requested in v): sum, aggregate store, split, nb
    auto consume = [&](int j, int beg, int end, int idl, v4f (&v)[G2_NB]) __attribute__((always_inline)) {
        const int B = j & 1;
        v4f acc{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < G2_NB; ++e) acc += v[e];
        const int deg = end - beg;
        // (rare: rows with more than G2_NB neighbours -- one round trip per
        // 16 more; ids past 32 read here)
        const int dmax = __builtin_amdgcn_readfirstlane(__float_as_int(wave_max(__int_as_float(deg))));
        for (int e0 = G2_NB; e0 < dmax; e0 += G2_NB) {
            const int il = (e0 & 31) == 0 ? ids_of(beg, end, e0) : idl;
            idl = il;
            rows_of(beg, end, e0, il, v);
#pragma unroll
            for (int e = 0; e < G2_NB; ++e) acc += v[e];
        }
        if (a.mean) {
            const float dv = static_cast<float>(deg > 1 ? deg : 1);
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i] = acc[i] / dv;
        }
        const int r = tile_row(j, srow);
        buf_store4(acc, ar, (r < n_rows && scol && !(DBG & 4)) ? r * static_cast<int>(a.ld_agg) * 4 + 16 * sslot : kOOB2, 0, 0);
        {  // parts of the tile row (max over the row's 32 lanes)
            const int e = h2_exp(max_xor16(max_row16(amax4(acc))));
            const v4f vs = ldexp4(acc, e);
            half4 p1, p2;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const _Float16 hh = static_cast<_Float16>(vs[i]);
                p1[i] = hh;
                p2[i] = static_cast<_Float16>(vs[i] - static_cast<float>(hh));
            }
            if (sslot < 8 * C0) {
                _Float16 *d = sxp + B * XPB + srow * PSTR + 4 * sslot;
                *reinterpret_cast<half4 *>(d) = p1;
                *reinterpret_cast<half4 *>(d + F2_ROWS * PSTR) = p2;
            }
            if (sslot == 0) serow[B * F2_ROWS + srow] = e;
        }
    };
    auto multiply = [&](int j, const half8 (&wl)[2][C0][2], int eW) __attribute__((always_inline)) {
        if (DBG & 2) return;
        const int B = j & 1;
        v4f o[2] = {v4f{0.f, 0.f, 0.f, 0.f}, v4f{0.f, 0.f, 0.f, 0.f}};
        const _Float16 *xp = sxp + B * XPB + rl * PSTR + 8 * q;
#pragma unroll
        for (int c = 0; c < C0; ++c) {
            const half8 x1 = *reinterpret_cast<const half8 *>(xp + 32 * c);
            const half8 x2 = *reinterpret_cast<const half8 *>(xp + F2_ROWS * PSTR + 32 * c);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) o[mt] = mfma_h2(wl[mt][c][0], wl[mt][c][1], x1, x2, o[mt]);
        }
        const int un = -(eW + serow[B * F2_ROWS + rl]);
        const int r2 = tile_row(j, rl);
        const int no = r2 < a.cap_rows ? r2 * F2_HID * 4 + (32 * wv + 4 * q) * 4 : kOOB2;
        buf_store4(ldexp4(o[0], un), nr, no, 0, 0);
        buf_store4(ldexp4(o[1], un), nr, no == kOOB2 ? kOOB2 : no + 64, 0, 0);
    };

    // prologue: row pointers of tiles 0..2, ids of 0..1, rows of tile 0 --
    // then this wave's W_l0 slice while they are in flight
    // (issue order: the index words, the weight slice, then tile 0's rows --
    // so the slice is split while the rows are in flight, and waiting for
    // tile 0's ids does not wait for the slice)
    int b0, e0, b1, e1, b2, e2;
    rowptr_of(0, b0, e0);
    rowptr_of(1, b1, e1);
    int i0 = ids_of(b0, e0, 0);
    rowptr_of(2, b2, e2);
    int i1 = ids_of(b1, e1, 0);
    v4f wt[2][C0][2];
    __builtin_amdgcn_sched_barrier(0);  // (keep the issue order: the scheduler hoists loads)
    if (!(DBG & 16)) w0_slice_issue<C0>(a.wl0, a.ldw0, a.K0, wv, ln, wt);
    __builtin_amdgcn_sched_barrier(0);
    v4f va[G2_NB], vb[G2_NB];
    rows_of(b0, e0, 0, i0, va);
    half8 wl[2][C0][2];
    int eW = 0;
    if (DBG & 16) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int c = 0; c < C0; ++c) wl[mt][c][0] = wl[mt][c][1] = half8{};
    } else {
        eW = w0_slice_finish<C0>(wt, wl);
    }
    if (DBG & 8) {  // (profiling: the prologue alone)
        if (va[0][0] == 1.2345f && wl[0][0][0][0] == static_cast<_Float16>(1.0f)) a.nb[0] = 0.0f;
        return;
    }

    // one step: request rowptr(j+3), ids(j+2), rows(j+1) into vn; consume
    // tile j from vc
    auto step = [&](int j, v4f (&vc)[G2_NB], v4f (&vn)[G2_NB]) __attribute__((always_inline)) {
        int b3, e3;
        rowptr_of(j + 3, b3, e3);
        const int i2 = ids_of(b2, e2, 0);
        rows_of(b1, e1, 0, i1, vn);
        consume(j, b0, e0, i0, vc);
        lds_barrier();
        multiply(j, wl, eW);
        b0 = b1; e0 = e1; i0 = i1;
        b1 = b2; e1 = e2; i1 = i2;
        b2 = b3; e2 = e3;
    };
    // (pairs of steps with ONE exit: at the back edge the tile in flight is
    // in va on every path, so the wait counters stay exact there; an odd
    // tail runs after the loop.  Requests past the last tile read nothing.)
    const int npair = ntj >> 1;
    for (int jj = 0; jj < npair; ++jj) {
        step(2 * jj, va, vb);
        step(2 * jj + 1, vb, va);
    }
    if (ntj & 1) step(ntj - 1, va, vb);
}

template <int C0, int DBG = 0>
__global__ __launch_bounds__(F2_WAVES * 64) void k_edge_nb(G2Args a) {
    edge_nb_body<C0, DBG>(a);
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
    const float *wr0;  // [256, K0], row stride ldw0
    int64_t ldw0;
    const float *wr1, *wl1;  // [F1, 256], row stride ldw1
    int64_t ldw1;
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
// the fused x[n_id] gather (rows through n_id, whose loads run four tiles
// ahead of the row loads that use them).  T16: K0 <= 32 C0 - 16 -- the last
// 32-deep chunk of layer 0 runs as a 16-deep one on v_mfma_f32_16x16x16_f16
// (K0 = 100: 3 x 32 + 16 instead of 4 x 32 -- an eighth of the launch's
// MFMA work and 8 weight registers).
// DBG (profiling builds only, NGNN_FWD2_DBG): bit 0 skips the reduce, 1 the
// layer-1 products, 2 layer 0's products, 3 the x split, 4 the out / z
// stores (offsets out of range), 5 the consumer's h reads (register
// operands), 6 the consumer's products (reads kept) -- time attribution
// ROOT false (ABI 17: wr0 NULL -- GCNConv's aggregate-first layer, W_r = 0):
// no x rows at all -- no loads, no split, no layer-0 products; h = act(b0 +
// nb) (act(b0) on rows without in-edges)
template <int C0, int NT1, int DM, bool XR, bool T16, int DBG = 0, bool ROOT = true>
__device__ __forceinline__ void fwd2_body(const F2Args &a) {
    static_assert(NT1 == 3, "layer 1's six output m-tiles map onto the waves (one each, two duplicates)");
    constexpr int CF = T16 ? C0 - 1 : C0;    // full 32-deep chunks of layer 0
    constexpr int KC = 32 * CF + (T16 ? 16 : 0);  // K0 padded to the chunks
    constexpr int PSTR = 32 * C0 + 16;       // halves per parts row: 72 dwords = 8 mod 64 banks (conflict-free fragment reads)
    constexpr int XPB = 2 * F2_ROWS * PSTR;  // halves per x-parts buffer (2 parts)
    constexpr int NK1 = F2_HID / 32;         // layer 1's 32-deep K chunks = the waves that produce h
    extern __shared__ __attribute__((aligned(16))) v4f lds2[];
    // h of a tile as layer 1's B fragments: [2 buffers][8 chunks (= producer
    // waves)][2 parts][64 lanes] half8 -- the producer's lane (q, rl) holds
    // exactly the fragment lane (q, rl) of a consumer reads (16-B, contiguous)
    half8 *shp = reinterpret_cast<half8 *>(lds2);                        // [2][8][2][64]
    _Float16 *sxp = reinterpret_cast<_Float16 *>(lds2 + 2 * NK1 * 2 * 64);  // [2][2][16][PSTR]
    int *serow = reinterpret_cast<int *>(sxp + 2 * XPB);                // [2][16]
    float *sb0 = reinterpret_cast<float *>(serow + 2 * F2_ROWS);        // [256] b0
    float *sb1 = sb0 + F2_HID;                                          // [16 NT1] b1 (0 past F1)
    float *sout = sb1 + 16 * NT1;                                       // [2][16 F1] out tiles, packed rows
    int *se1 = reinterpret_cast<int *>(sout + 2 * F2_ROWS * 16 * NT1);  // [2][16][8] h-chunk exponents (row, chunk)
    float *strash = reinterpret_cast<float *>(se1 + 2 * F2_ROWS * F2_WAVES);  // [64] sink of the lanes with nothing to write
    static_assert(PSTR >= 128, "the split's lanes 4 sslot + 3 < 128 write inside a parts row");

    const int wv = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int ln = threadIdx.x & 63, q = ln >> 4, rl = ln & 15;
    // the biases in LDS (read per tile: registers are the scarce resource here).
    // Bit-mode dropout (DM 2) keeps with the exact scale 2: b0, the unscale
    // and nb carry that factor (2 (acc s + b0) + 2 nb rounds as acc 2s + 2 b0
    // + 2 nb: scaling by two commutes with rounding), so the epilogue has no
    // multiply
    if (threadIdx.x < F2_HID) sb0[threadIdx.x] = DM == 2 ? 2.0f * a.b0[threadIdx.x] : a.b0[threadIdx.x];
    if (threadIdx.x < 16 * NT1) sb1[threadIdx.x] = static_cast<int>(threadIdx.x) < a.F1 ? a.b1[threadIdx.x] : 0.0f;
    // ---- this wave's weight slices, for the whole launch
    half8 wr[2][CF][2], w1[NK1][2];
    half4 wt[2][2];  // T16: the tail chunk, k = 32 CF + 4 q .. + 3
    int eW0 = 0;
    if constexpr (ROOT) {
        v4f t[2][CF][2], tt[2];
        w0_slice_issue<CF>(a.wr0, a.ldw0, a.K0, wv, ln, t);
        if (T16) {
            const i32x4 wrs = make_rsrc(a.wr0, static_cast<uint32_t>(static_cast<int64_t>(F2_HID) * a.ldw0 * 4));
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                const int k = 32 * CF + 4 * q;
                tt[mt] = buf_load4(wrs, k < a.K0 ? (32 * wv + 16 * mt + rl) * static_cast<int>(a.ldw0) * 4 + 4 * k : kOOB2, 0, 0);
            }
        }
        float mx = 0.0f;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
            for (int c = 0; c < CF; ++c) mx = fmaxf(mx, fmaxf(amax4(t[mt][c][0]), amax4(t[mt][c][1])));
            if (T16) mx = fmaxf(mx, amax4(tt[mt]));
        }
        eW0 = __builtin_amdgcn_readfirstlane(h2_exp(wave_max(mx)));
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
            for (int c = 0; c < CF; ++c) h2_split(ldexp4(t[mt][c][0], eW0), ldexp4(t[mt][c][1], eW0), wr[mt][c][0], wr[mt][c][1]);
            if (T16) {
                const v4f v = ldexp4(tt[mt], eW0);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const _Float16 hh = static_cast<_Float16>(v[i]);
                    wt[mt][0][i] = hh;
                    wt[mt][1][i] = static_cast<_Float16>(v[i] - static_cast<float>(hh));
                }
            }
        }
    }
    // Layer 1 without a cross-wave reduction (round 6).  The six output
    // m-tiles of [W_r1 | W_l1] (out's 48 columns, then z's) go to six waves,
    // each over ALL 256 of layer 1's K: out waves 0, 1, 3 take W_r1's m-tiles
    // 0, 1, 2 and z waves 4, 5, 6 W_l1's (SIMD partners w, w + 4: two
    // consumers on SIMDs 0 and 1, one on 2 and 3); waves 2 and 7 repeat m-tile
    // 2 and store nothing (uniform code, the pipeline keeps its two
    // instantiations).  Every wave still produces 32 columns of h: it splits
    // them as before (its own per-row exponent) and leaves the two fp16 parts
    // in LDS as B fragments; a consumer runs the 8 chunks, rescaling its
    // accumulator by the exponent step between chunks (an exact power of two
    // per lane: a lane's 4 accumulator values share one tile row).
    // The wave's slice: output rows 16 mt1 + rl, K = 32 c + (4 q + j, 16 + 4 q + j)
    // for chunk c -- the order of producer c's lane (q, rl) values of h.
    const int l1z = wv >= F2_WAVES / 2;                   // z (W_l1) or out (W_r1)
    const int mt1 = min(wv & 3, NT1 - 1);                 // this wave's output m-tile
    const bool l1dup = wv == 2 || wv == F2_WAVES - 1;     // duplicates: nothing stored
    int eW1;
    {
        // (buffer loads, counted in order with the kernel's other loads)
        v4f t[NK1][2];
        float mx = 0.0f;
        const i32x4 w1r = make_rsrc(l1z ? a.wl1 : a.wr1, static_cast<uint32_t>(a.F1 * a.ldw1 * 4));
        const int o = 16 * mt1 + rl;
        const int rb = o < a.F1 ? o * static_cast<int>(a.ldw1) * 4 : kOOB2;
#pragma unroll
        for (int c = 0; c < NK1; ++c) {
            const int c0 = (32 * c + 4 * q) * 4, c1 = (32 * c + 16 + 4 * q) * 4;
            t[c][0] = buf_load4(w1r, rb == kOOB2 ? kOOB2 : rb + c0, 0, 0);
            t[c][1] = buf_load4(w1r, rb == kOOB2 ? kOOB2 : rb + c1, 0, 0);
        }
#pragma unroll
        for (int c = 0; c < NK1; ++c) mx = fmaxf(mx, fmaxf(amax4(t[c][0]), amax4(t[c][1])));
        eW1 = __builtin_amdgcn_readfirstlane(h2_exp(wave_max(mx)));
#pragma unroll
        for (int c = 0; c < NK1; ++c) h2_split(ldexp4(t[c][0], eW1), ldexp4(t[c][1], eW1), w1[c][0], w1[c][1]);
    }
    // out: its rows are F1 floats wide (188 B, not 16-B aligned), but a
    // tile's 16 rows are ONE contiguous 16-B-aligned block of 64 F1 bytes --
    // the sums go to an LDS staging tile in that packed order and leave, a
    // step later, as contiguous 16-B stores (dword stores scattered over 16
    // rows cost a third of the kernel).  z: one 16-B store a lane.  One store
    // instruction per wave and step either way.  The consumer lane (q, rl)
    // holds output columns 16 mt1 + 4 q .. + 3 of tile row rl.
    const int rzt = l1z;
    const int rcol = 16 * mt1 + 4 * q;  // first output column of the lane
    // the duplicates' (and out's past-F1 columns') sinks as lane values the
    // compiler cannot branch on: a wave-uniform test inside a step made it
    // split the step into blocks with scalar and exec branches
    // (one register: bits 0-3 -- column rcol + i of out goes to the sink;
    // bits 28-31 -- kOOB2, OR-ed into a duplicate's z store offset)
    int lsink = l1dup ? kOOB2 : 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) lsink |= (l1dup || rcol + i >= a.F1) ? 1 << i : 0;
    asm volatile("" : "+v"(lsink));
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
    const i32x4 zrs = make_rsrc(a.z, static_cast<uint32_t>(static_cast<int64_t>(n_rows) * a.ldz * 4));
    const i32x4 ors = make_rsrc(a.out, static_cast<uint32_t>(static_cast<int64_t>(n_rows) * a.F1 * 4));
    const int F1 = a.F1;
    const uint32_t ld4 = static_cast<uint32_t>(a.ldx) * 4u;

    // ---- x split lanes: row srow of the tile, columns 4 sslot .. + 3
    const int srow = 2 * wv + (ln >> 5), sslot = ln & 31;
    const bool scol = 4 * sslot < a.K0 && 4 * sslot < KC;
    auto tile_of = [&](int j) { return b + j * G; };
    // XR: the split row's feature-table index (low word of n_id; rows past
    // the block read 0 and are masked at use)
    auto iload = [&](int j) __attribute__((always_inline)) -> int {
        if constexpr (!ROOT) return 0;
        const int row = tile_of(j) * F2_ROWS + srow;
        return buf_load1i(ir, row < n_rows ? row * 8 : kOOB2, 0, 0);
    };
    auto xload = [&](int j, int idx) __attribute__((always_inline)) -> v4f {
        if constexpr (!ROOT) return v4f{0.f, 0.f, 0.f, 0.f};
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
        if constexpr (!ROOT) return;
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
        // (no branches in a step: the lanes past KC write zeros into the row's
        // padding, the row's other 31 lanes their exponent into the sink)
        _Float16 *d = sxp + buf * XPB + srow * PSTR + 4 * sslot;
        *reinterpret_cast<half4 *>(d) = p1;
        *reinterpret_cast<half4 *>(d + F2_ROWS * PSTR) = p2;
        int *ed = sslot == 0 ? serow + buf * F2_ROWS + srow : reinterpret_cast<int *>(strash) + ln;
        *ed = e;
    };
    // layer 0's products of one tile (its parts buffer), this wave's 32
    // columns; s0 = the lane row's unscale 2^-(eW0 + e_row) (read here: the
    // buffer's exponents are overwritten in the next step)
    auto l0 = [&](int buf, v4f (&acc)[2], float &s0) __attribute__((always_inline)) {
        acc[0] = v4f{0.f, 0.f, 0.f, 0.f};
        acc[1] = v4f{0.f, 0.f, 0.f, 0.f};
        if constexpr (!ROOT) {
            s0 = 0.0f;  // (b0 + nb alone: fma(0, 0, b0) = b0)
            return;
        }
        const _Float16 *xp = sxp + buf * XPB + rl * PSTR + 8 * q;
        half8 xf[CF][2];  // every fragment read issued before the first MFMA
        half4 xt[2];
#pragma unroll
        for (int c = 0; c < CF; ++c) {
            xf[c][0] = *reinterpret_cast<const half8 *>(xp + 32 * c);
            xf[c][1] = *reinterpret_cast<const half8 *>(xp + F2_ROWS * PSTR + 32 * c);
        }
        if (T16) {  // (16x16x16: lane (q, rl) holds k = 4 q .. + 3 of row rl)
            xt[0] = *reinterpret_cast<const half4 *>(xp - 4 * q + 32 * CF);
            xt[1] = *reinterpret_cast<const half4 *>(xp - 4 * q + 32 * CF + F2_ROWS * PSTR);
        }
        s0 = __builtin_amdgcn_ldexpf(1.0f, (DM == 2 ? 1 : 0) - (eW0 + serow[buf * F2_ROWS + rl]));
#pragma unroll
        for (int c = 0; c < CF; ++c)
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) acc[mt] = mfma_h2(wr[mt][c][0], wr[mt][c][1], xf[c][0], xf[c][1], acc[mt]);
        if (T16) {
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                acc[mt] = __builtin_amdgcn_mfma_f32_16x16x16f16(wt[mt][1], xt[0], acc[mt], 0, 0, 0);
                acc[mt] = __builtin_amdgcn_mfma_f32_16x16x16f16(wt[mt][0], xt[1], acc[mt], 0, 0, 0);
                acc[mt] = __builtin_amdgcn_mfma_f32_16x16x16f16(wt[mt][0], xt[0], acc[mt], 0, 0, 0);
            }
        }
    };
    // one tile after layer 0: epilogue, h rows, h's layer-1 fragments into shp[buf]
    auto finish = [&](int j, int buf, const v4f (&acc)[2], float s0, const v4f (&nbv)[2], auto nb_c)
        __attribute__((always_inline)) {
        constexpr bool NB = decltype(nb_c)::value;
        const int r = tile_of(j) * F2_ROWS + rl;
        // b0 + x W_r0^T (+ nb), ReLU (NaN passes), dropout keyed by (global
        // row, global column) exactly as every other forward kernel.  The
        // unscale rides the fma (acc s0 is exact: a power of two)
        const uint32_t rk = DM ? drop.row_key(static_cast<uint32_t>(r)) : 0u;
        // columns 32 wv .. + 31; the lane's bits 16 mt + 4 q + i, shifted by 4 q
        // once so the per-value shifts are immediates
        const uint32_t hw = DM == 2 ? lowbias32(rk + static_cast<uint32_t>(wv)) >> (4 * q) : 0u;
        v4f hv[2], b0v[2];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) b0v[mt] = *reinterpret_cast<const v4f *>(sb0 + 32 * wv + 16 * mt + 4 * q);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            const uint32_t hq = DM == 1 ? lowbias32(rk + static_cast<uint32_t>(8 * wv + 4 * mt + q)) : 0u;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float y = __builtin_fmaf(acc[mt][i], s0, b0v[mt][i]);
                if (NB) y = DM == 2 ? __builtin_fmaf(nbv[mt][i], 2.0f, y) : y + nbv[mt][i];
                if (DM == 1) {
                    const bool zero = y < 0.0f || ((hq >> (8 * i)) & 0xffu) < drop.thresh;
                    hv[mt][i] = zero ? 0.0f : y * drop.scale;
                } else {
                    // ReLU and the keep bit as bit masks (three VALU ops):
                    // y & ~sign(y) & keep -- +NaN passes, -NaN and -0 give +0
                    const int yb = __float_as_int(y);
                    int m = ~(yb >> 31);
                    if (DM == 2) m &= __builtin_amdgcn_sbfe(static_cast<int>(hw), 16 * mt + i, 1);
                    hv[mt][i] = __int_as_float(yb & m);
                }
            }
        }
        // h rows the backward reads (past the bound: dropped by the range)
        const int ho = static_cast<int>(static_cast<uint32_t>(r) * static_cast<uint32_t>(a.ldh) * 4u) + (32 * wv + 4 * q) * 4;
        buf_store4(hv[0], hrs, r < hr ? ho : kOOB2, 0, NGNN_F2_STAUX_H);
        buf_store4(hv[1], hrs, r < hr ? ho + 64 : kOOB2, 0, NGNN_F2_STAUX_H);
        // layer 1's chunk wv of K: the lane's own 8 values of h ARE the B
        // fragment lane (q, rl) of that chunk (k order 4q + i, 16 + 4q + i),
        // split after scaling by the row's exponent over this wave's 32
        // columns.  h >= +0 (or +NaN): its bit patterns order as ints
        int mb = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) mb = max(mb, __float_as_int(i < 4 ? hv[0][i] : hv[1][i - 4]));
        const float m = max_xor32(max_xor16(__int_as_float(mb)));  // lanes rl + 16 q
        const int eh = h2_exp(m);
        half8 h1, h2;
        h2_split(ldexp4(hv[0], eh), ldexp4(hv[1], eh), h1, h2);
        if (DBG & 2) {
            asm volatile("" : "+v"(h1), "+v"(h2));
            return;
        }
        // both parts to LDS (two contiguous 1-KiB wave stores), the row's
        // exponent from lane q = 0 (the row's other lanes into the sink)
        half8 *hd = shp + (buf * NK1 + wv) * 2 * 64 + ln;
        hd[0] = h1;
        hd[64] = h2;
        int *ed = q == 0 ? se1 + (buf * F2_ROWS + rl) * F2_WAVES + wv : reinterpret_cast<int *>(strash) + ln;
        *ed = eh;
    };
    // the 8 partials of this lane's item, summed in wave order (+ b1), stored
    // (jj < 0: the step before the first tile -- nothing live)
    // reduce(jj): the summed partials of tile jj -- out waves stage them in
    // sout[jj & 1] (+ b1), z waves keep them for their store
    // (RZ: a z wave -- waves 4-7, the LAG half; compile-time inside the
    // pipeline, so a step has no branches).  The partials are unscaled here,
    // in the fma that sums them (wave order, as a sum of the exact products)
    // layer1(jj): this wave's output m-tile of tile jj from the 8 producers'
    // h fragments -- out waves add b1 and stage it in sout[jj & 1], z waves
    // keep it for their store.  Chunk c's products carry the scale 2^(eW1 +
    // e_c) (e_c: producer c's exponent of the lane's row); the accumulator is
    // moved to chunk c's scale before its products (exact: a power of two),
    // in two chains (even / odd chunks) so an MFMA result is not waited on at
    // every chunk, and both chains are unscaled exactly at the end.
    auto reduce = [&](int jj, int buf, auto z_c) __attribute__((always_inline)) -> v4f {
        constexpr bool RZ = decltype(z_c)::value;
        const int *ep = se1 + (buf * F2_ROWS + rl) * F2_WAVES;
        const i32x4 ea = *reinterpret_cast<const i32x4 *>(ep), eb = *reinterpret_cast<const i32x4 *>(ep + 4);
        const half8 *hp = shp + buf * NK1 * 2 * 64 + ln;
        v4f acc[2] = {v4f{0.f, 0.f, 0.f, 0.f}, v4f{0.f, 0.f, 0.f, 0.f}};
        // the fragments two chunks ahead of their MFMAs (a 2-slot ring: the
        // compiler, left alone, hoisted all 16 reads -- 64 registers -- and
        // spilled)
        half8 bf[2][2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if (DBG & 32) {  // (profiling: no h reads -- register operands)
                bf[c][0] = w1[c][0];
                bf[c][1] = w1[c][1];
                asm volatile("" : "+v"(bf[c][0]), "+v"(bf[c][1]));
                continue;
            }
            bf[c][0] = hp[2 * c * 64];
            bf[c][1] = hp[(2 * c + 1) * 64];
        }
#pragma unroll
        for (int c = 0; c < NK1; ++c) {
            const half8 b1 = bf[c & 1][0], b2 = bf[c & 1][1];
            if (c >= 2) {
                const int ep2 = c - 2 < 4 ? ea[c - 2] : eb[c - 6];
                const int ec = c < 4 ? ea[c] : eb[c - 4];
                acc[c & 1] *= __builtin_amdgcn_ldexpf(1.0f, ec - ep2);  // scale 2^(eW1 + e_{c-2}) -> 2^(eW1 + e_c)
            }
            if (DBG & 64) {  // (profiling: the h reads without the products)
                asm volatile("" : "+v"(acc[c & 1]) : "v"(b1), "v"(b2));
            } else {
                acc[c & 1] = mfma_h2(w1[c][0], w1[c][1], b1, b2, acc[c & 1]);
            }
            if (c + 2 < NK1) {
                if (DBG & 32) {
                    bf[c & 1][0] = w1[c + 2][0];
                    bf[c & 1][1] = w1[c + 2][1];
                    asm volatile("" : "+v"(bf[c & 1][0]), "+v"(bf[c & 1][1]));
                } else {
                    bf[c & 1][0] = hp[2 * (c + 2) * 64];
                    bf[c & 1][1] = hp[(2 * (c + 2) + 1) * 64];
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        v4f s = acc[0] * __builtin_amdgcn_ldexpf(1.0f, -(eW1 + eb[2]));
        s += acc[1] * __builtin_amdgcn_ldexpf(1.0f, -(eW1 + eb[3]));
        if (!RZ) {
            s += *reinterpret_cast<const v4f *>(sb1 + rcol);
            // (columns past F1 and the duplicate wave into the sink: no two
            // lanes of one ds_write on the same dword)
            float *d = sout + (jj & 1) * F2_ROWS * F1 + rl * F1 + rcol;
#pragma unroll
            for (int i = 0; i < 4; ++i) *(((lsink >> i) & 1) ? strash + ln : d + i) = s[i];
        }
        return s;
    };
    // ONE 16-B store per wave: z waves the z item of tile jz (sum s), out
    // waves piece p = threadIdx.x of the staged out tile jo (sout[jo & 1]:
    // tile jo's 16 rows are 4 F1 contiguous 16-B pieces of out)
    auto store = [&](int jz, v4f s, int jo, auto z_c) __attribute__((always_inline)) {
        constexpr bool RZ = decltype(z_c)::value;
        if (RZ) {
            const int zrow = tile_of(jz) * F2_ROWS + rl;
            const int zo = ((jz >= 0 && zrow < n_rows)
                                ? static_cast<int>(static_cast<uint32_t>(zrow) * static_cast<uint32_t>(a.ldz) * 4u) + 4 * rcol
                                : kOOB2) | (lsink & kOOB2);
            buf_store4(s, zrs, (DBG & 16) ? kOOB2 : zo, 0, NGNN_F2_STAUX_Z);
        } else {
            const int p = static_cast<int>(threadIdx.x);  // (out waves: < 256)
            const v4f v = *reinterpret_cast<const v4f *>(sout + (jo & 1) * F2_ROWS * F1 + 4 * min(p, 4 * F1 - 1));
            const int oo = (jo >= 0 && p < 4 * F1) ? tile_of(jo) * F2_ROWS * F1 * 4 + 16 * p : kOOB2;
            buf_store4(v, ors, (DBG & 16) ? kOOB2 : oo, 0, NGNN_F2_STAUX_O);
        }
    };
    // the workgroup's last tile jo, which may end inside a piece (n_rows not
    // a multiple of 16): element stores for that piece
    auto out_store_last = [&](int jo) __attribute__((always_inline)) {
        if (rzt) return;
        const int p = static_cast<int>(threadIdx.x);
        const v4f v = *reinterpret_cast<const v4f *>(sout + (jo & 1) * F2_ROWS * F1 + 4 * min(p, 4 * F1 - 1));
        const int base = tile_of(jo) * F2_ROWS * F1 * 4;
        const int nv = min(n_rows - tile_of(jo) * F2_ROWS, F2_ROWS) * F1;  // valid elements of the tile
        if (4 * p + 4 <= nv) {
            buf_store4(v, ors, base + 16 * p, 0, 0);
        } else if (4 * p < nv) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (4 * p + i < nv) buf_store1(v[i], ors, base + 16 * p + 4 * i, 0, 0);
        }
    };

    // ---- software pipeline over the workgroup's tiles.  Step j:
    //   reduce(j - 1)  -- layer 1 of the previous tile (shp[(j-1)&1]: MFMA)
    //   l0(j + 1)      -- MFMA on parts buffer (j+1)&1 (split last step)
    //   finish(j)      -- VALU epilogue + h split -> shp[j&1]
    //   split(j + 2)   -- x rows from the register ring -> parts buffer j&1
    //   ONE barrier
    // so every step holds independent MFMA and VALU work for the scheduler
    // (layer 0 of the next tile beside the epilogue of this one).  Buffer
    // safety: parts buffer j&1 was last read by l0(j) in step j - 1, shp
    // (j-1)&1 is rewritten in step j + 1 -- each behind a barrier.
    //
    // x rows are loaded two steps before their split (a 2-slot register ring).
    // vmcnt counts vector-memory ops IN ORDER, so a load consumed soon after
    // its issue forces every older one -- the x prefetches -- to land with
    // it.  Hence: the edge tiles (nb loaded one tile ahead, first in the
    // step) run in a phase of their own; XR's n_id loads run two steps ahead
    // of the row loads that use them; loads pending at a phase entry are
    // SETTLED first (the compiler's wait for a loop-carried load takes the
    // fewest younger memory ops over the paths into the loop); the loops have
    // no exits between steps.
    // the whole pipeline, instantiated twice: LAG (waves 4-7) runs each step's
    // two halves in the other order (MI355X_MICROARCH.md: stagger SIMD
    // partners by wave number >= 4)
    auto pipeline = [&](auto lag_c) __attribute__((always_inline)) {
        constexpr bool LAG = decltype(lag_c)::value;
#ifdef NGNN_F2_SETPRIO
        // (A/B: static priority for the second-dispatched half, waves 4-7 --
        // MI355X_MICROARCH.md, scheduling item 4)
        if (LAG) __builtin_amdgcn_s_setprio(1);
#endif
        // x ring: at step j, xv[j&1] holds tile j + 2 and xv[~j&1] tile j + 3;
        // XR: ixr[j&1] holds n_id of tile j + 4
        v4f xv[2];
        int ixr[2] = {0, 0};
        xv[0] = xload(0, XR ? iload(0) : 0);
        xv[1] = xload(1, XR ? iload(1) : 0);
        v4f nbv[2];  // nb of the tile the next finish() takes (edge phase)
        nbload(0, nbv);
        split(xv[0], 0);
        split(xv[1], 1);
        xv[0] = xload(2, XR ? iload(2) : 0);
        xv[1] = xload(3, XR ? iload(3) : 0);
        if (XR) {
            ixr[0] = iload(4);
            ixr[1] = iload(5);
        }
        auto settle = [&]() __attribute__((always_inline)) {
            asm volatile("" : "+v"(xv[0]), "+v"(xv[1]), "+v"(ixr[0]), "+v"(ixr[1]));
            asm volatile("" : "+v"(nbv[0]), "+v"(nbv[1]));
        };
        settle();
        lds_barrier();
        v4f acc[2];
        float s0;
        l0(0, acc, s0);
        lds_barrier();  // (every wave's reads of parts buffer 0 before step 0 rewrites it)
        const v4f zz[2] = {v4f{0.f, 0.f, 0.f, 0.f}, v4f{0.f, 0.f, 0.f, 0.f}};
        auto step = [&](auto u_c, auto nb_c, int j) __attribute__((always_inline)) {
            constexpr int U = decltype(u_c)::value;     // j % 4
            constexpr int B = U & 1;                    // j % 2
            constexpr bool NB = decltype(nb_c)::value;  // an edge-tile phase
            v4f accn[2];
            float s0n;
            // front: layer 0 of the next tile (fragment reads + MFMA), then the
            // reduce (LDS reads) and the store
            auto front = [&]() __attribute__((always_inline)) {
                if (!(DBG & 4)) {
                    l0(B ^ 1, accn, s0n);
                } else {
                    accn[0] = xv[0];
                    accn[1] = xv[1];
                    s0n = 1.0f;  // (DBG only)
                }
                if (!(DBG & 1)) {
                    // z of tile j - 1 / out of tile j - 2 (staged in step j - 1;
                    // the buffers differ from this step's staging writes)
                    const v4f rs = reduce(j - 1, B ^ 1, lag_c);
                    store(j - 1, rs, j - 2, lag_c);
                }
            };
            // back: the VALU-heavy epilogue + layer-1 products, the split, the loads
            auto back = [&]() __attribute__((always_inline)) {
                finish(j, B, acc, s0, NB ? nbv : zz, nb_c);
                if (!(DBG & 8)) {
                    split(xv[B], B);  // tile j + 2
                } else {
                    asm volatile("" : "+v"(xv[B]));
                }
                // nb of the next tile BEFORE the x load: its wait next step leaves
                // the younger x loads in flight
                if (NB) nbload(j + 1, nbv);
                xv[B] = xload(j + 4, ixr[B]);
                if (XR) ixr[B] = iload(j + 6);
            };
            // (the halves are independent within a step; SIMD partners -- waves
            // w and w + 4 -- run them in opposite orders, so one's MFMAs meet the
            // other's VALU instead of both stalling on the same phase)
            // The halves stay apart (sched_barrier): left to interleave them,
            // the scheduler's order measured 84.3 vs 82.7 us per launch
            if (!LAG) {
                front();
                __builtin_amdgcn_sched_barrier(0);
                back();
            } else {
                back();
                __builtin_amdgcn_sched_barrier(0);
                front();
            }
            lds_barrier();
            acc[0] = accn[0];
            acc[1] = accn[1];
            s0 = s0n;
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
        bool done = false;
        for (; j < ntj_e; j += 4) {
            step(I0{}, std::true_type{}, j);
            if (j + 1 >= ntj) { done = true; break; }
            step(I1{}, std::true_type{}, j + 1);
            if (j + 2 >= ntj) { done = true; break; }
            step(I2{}, std::true_type{}, j + 2);
            if (j + 3 >= ntj) { done = true; break; }
            step(I3{}, std::true_type{}, j + 3);
        }
        if (!done && j < ntj) {
            settle();  // (the x rows in flight: settled once at the phase change)
            // whole trips of 4 steps with no exits inside, then the remainder
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
        if (!(DBG & 1)) {
            // z of the last tile, out of tile ntj - 2 (staged before the last
            // barrier); then the last tile's out: staged, one more barrier
            const v4f rs = reduce(ntj - 1, (ntj - 1) & 1, lag_c);
            store(ntj - 1, rs, ntj - 2, lag_c);
            lds_barrier();
            out_store_last(ntj - 1);
        }
    };
    if (wv >= F2_WAVES / 2) pipeline(std::true_type{});
    else pipeline(std::false_type{});
}

template <int C0, int NT1, int DM, bool XR, bool T16, int DBG = 0, bool ROOT = true>
__global__ __launch_bounds__(F2_WAVES * 64) void k_fwd2(F2Args a) {
    fwd2_body<C0, NT1, DM, XR, T16, DBG, ROOT>(a);
}

// Both launches as ONE (round 5): the edge phase and the main phase map tile
// t to workgroup t % G alike, so the nb rows a workgroup's main phase reads
// are the ones its own edge phase wrote -- by the same lanes (k_edge_nb's
// multiply and k_fwd2's nbload address a row's columns 32 wv + 4 q .. alike)
// -- and the only hand-off is this workgroup's barrier.  Saves the launch
// boundary and lets workgroups with fewer edge tiles start their main tiles
// while others still gather (the edge phase has ~4 tiles per workgroup on
// the products block, the main phase ~38).  The edge phase's LDS is static,
// the main phase's dynamic: both fit together (138 KB).
template <int C0, int NT1, int DM, bool XR, bool T16, bool ROOT = true>
__global__ __launch_bounds__(F2_WAVES * 64) void k_fwd2x(G2Args g, F2Args f) {
    edge_nb_body<C0, 0>(g);
    __syncthreads();  // (workgroup scope: this workgroup's nb / agg stores before its main phase's reads)
    fwd2_body<C0, NT1, DM, XR, T16, 0, ROOT>(f);
}

template <int C0, int NT1, int DM, bool XR, int DBG = 0, bool T16 = false, bool ROOT = true>
int launch_fwd2(const F2Args &a, int grid, hipStream_t st) {
    auto fn = k_fwd2<C0, NT1, DM, XR, T16, DBG, ROOT>;
    const size_t lds = static_cast<size_t>(2) * (F2_HID / 32) * 2 * 64 * 16 +
                       static_cast<size_t>(2) * 2 * F2_ROWS * (32 * C0 + 16) * 2 + 2 * F2_ROWS * 4 +
                       (F2_HID + 16 * NT1) * 4 + 2 * F2_ROWS * 16 * NT1 * 4 + 2 * F2_ROWS * F2_WAVES * 4 + 64 * 4;
    static bool attr_set = false;  // benign race: idempotent
    if (!attr_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(F2_WAVES * 64), lds, st, a);
    return launch_status();
}

template <int C0, int NT1, int DM, bool XR, bool T16 = false, bool ROOT = true>
int launch_fwd2x(const G2Args &g, const F2Args &a, int grid, hipStream_t st) {
    auto fn = k_fwd2x<C0, NT1, DM, XR, T16, ROOT>;
    const size_t lds = static_cast<size_t>(2) * (F2_HID / 32) * 2 * 64 * 16 +
                       static_cast<size_t>(2) * 2 * F2_ROWS * (32 * C0 + 16) * 2 + 2 * F2_ROWS * 4 +
                       (F2_HID + 16 * NT1) * 4 + 2 * F2_ROWS * 16 * NT1 * 4 + 2 * F2_ROWS * F2_WAVES * 4 + 64 * 4;
    static bool attr_set = false;  // benign race: idempotent
    if (!attr_set) {
        // (the edge phase's static LDS counts against the same 160 KiB: the
        // dynamic maximum is exactly what the main phase takes -- a 160 KiB
        // request is refused, and the launch then fails)
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(fn),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
        if (e != hipSuccess) return static_cast<int>(e);
        attr_set = true;
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(F2_WAVES * 64), lds, st, g, a);
    return launch_status();
}

template <int C0, int DBG = 0>
int launch_edge_nb(const G2Args &a, int grid, hipStream_t st) {
    hipLaunchKernelGGL((k_edge_nb<C0, DBG>), dim3(grid), dim3(F2_WAVES * 64), 0, st, a);
    return launch_status();
}

// workspace layout (256-B aligned pieces)
struct Ws2 {
    size_t nb, z, total;
};
Ws2 ws2_layout(int64_t K0, int64_t F1, int64_t n_rows) {
    (void)K0;
    const int64_t NT1 = ceil_div(F1, 16);
    Ws2 w;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += (bytes + 255) & ~size_t(255);
        return o;
    };
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
                      const int32_t *n_edge_rows_dev, int reduce, float *out, int64_t ldo, hipStream_t st,
                      const NarrowHead *head);

}  // namespace ngnn

using namespace ngnn;

extern "C" int ngnn_sage2_supported(int64_t K0, int64_t H, int64_t F1, int reduce) {
    return (K0 > 96 && K0 <= 128 && K0 % 4 == 0 && H == F2_HID && F1 > 32 && F1 <= 48 &&
            (reduce == NGNN_REDUCE_MEAN || reduce == NGNN_REDUCE_SUM))
               ? 1
               : 0;
}

extern "C" size_t ngnn_xent_head_workspace_bytes(int64_t B) {
    // the top ticket and the label count, 32 group tickets (from byte 64),
    // then 32 group sums and one partial per workgroup holding seed rows (at
    // most B of them) from byte 256
    return B > 0 ? 256 + 4 * (32 + static_cast<size_t>(B)) : 0;
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
                              int64_t ldo, const ngnn_xent_head *head, int stages, void *ws, size_t ws_bytes,
                              void *stream) {
    NGNN_RETURN_IF(!ngnn_sage2_supported(K0, H, F1, reduce), NGNN_E_SHAPE);
    NGNN_RETURN_IF(n_rows < 0 || n_edge_rows < 0 || h_rows < 0, NGNN_E_ARG);
    NGNN_RETURN_IF(p_drop < 0.0f || !(p_drop <= 1.0f), NGNN_E_ARG);
    NGNN_RETURN_IF(stages <= 0 || stages > NGNN_SAGE2_ALL, NGNN_E_ARG);
    NGNN_RETURN_IF(ldx < K0 || ldx % 4 != 0 || ldw0 < K0 || ldw0 % 4 != 0 || ldw1 < H || ldw1 % 4 != 0 || ldh < H || ldh % 4 != 0 ||
                       ld_agg < K0 || ld_agg % 4 != 0 || ldo != F1,
                   NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(n_rows), NGNN_E_RANGE);
    const bool indexed = xrow || xrow_dev;
    NGNN_RETURN_IF(indexed && (x_rows <= 0 || !col_x), NGNN_E_ARG);
    if (n_rows == 0) return NGNN_OK;
    // (wr0 NULL, ABI 17: no root term -- GCNConv(normalize=False)'s layer;
    // not with the fused x[n_id] gather)
    NGNN_RETURN_IF(!wr0 && (xrow || xrow_dev), NGNN_E_ARG);
    NGNN_RETURN_IF((!x && !x_dev) || !rowptr || (!col && n_edge_rows > 0) || !wl0 || !bl0 || !wl1 || !bl1 || !wr1 ||
                       !h || !agg0 || !out || !ws,
                   NGNN_E_ARG);
    NGNN_RETURN_IF((x && !aligned(x, 16)) || !aligned(h, 16) || !aligned(out, 16) || !aligned(agg0, 16) || !aligned(bl0, 16) ||
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
    const int64_t C4 = (F1 + 3) & ~int64_t{3};
    if (head) {
        NGNN_RETURN_IF(!head->y || !head->loss || !head->count || !head->dy || !head->ws, NGNN_E_ARG);
        NGNN_RETURN_IF(head->B <= 0 || head->B > n_rows || head->ldd < F1, NGNN_E_ARG);
        NGNN_RETURN_IF(head->g && (head->g_rows < 0 || head->g_rows > n_rows), NGNN_E_ARG);
        NGNN_RETURN_IF(head->ws_bytes < ngnn_xent_head_workspace_bytes(head->B), NGNN_E_WORKSPACE);
        NGNN_RETURN_IF(!aligned(head->ws, 16) || (head->g && !aligned(head->g, 16)), NGNN_E_ALIGN);
        NGNN_RETURN_IF(head->g && head->g_rows * C4 * 4 > lim, NGNN_E_RANGE);
    }
    hipStream_t st = as_stream(stream);
    char *wsb = static_cast<char *>(ws);
    const int C0 = static_cast<int>(ceil_div(K0, 32)), NT1 = static_cast<int>(ceil_div(F1, 16));
    float *nb = reinterpret_cast<float *>(wsb + L.nb);
    float *z = reinterpret_cast<float *>(wsb + L.z);
    const int64_t ldz = 16 * NT1;
    const int64_t cap_rows = ceil_div(n_rows, 16) * 16;
    // the saved aggregate's and nb's rows: whole edge tiles (NB: agg0 must hold
    // ceil16(n_edge) rows when they exceed n_rows -- capped at n_rows here)
    // (NGNN_SAGE2_PREP: accepted, nothing to do -- the kernels load their
    // weight slices themselves since ABI 13's first release)
    const int ncu = num_cus();
    // the edge and main launches as one (k_fwd2x) when both run in this call
    // (NGNN_FWD2_FUSE=0, read once: two launches -- A/B)
    static const bool fuse_env = [] {
        const char *v = std::getenv("NGNN_FWD2_FUSE");
        return !(v && v[0] == '0');
    }();
    bool fuse = fuse_env && (stages & NGNN_SAGE2_MAIN) && (stages & NGNN_SAGE2_EDGE) && n_edge_rows > 0 &&
                C0 == 4 && NT1 == 3;
#ifdef NGNN_FWD2_DBG_BUILD
    if (getenv("NGNN_FWD2_DBG") || getenv("NGNN_EDGE_DBG")) fuse = false;
#endif
    G2Args g{};
    if ((stages & NGNN_SAGE2_EDGE) && n_edge_rows > 0) {
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
        g.wl0 = wl0;
        g.ldw0 = ldw0;
        g.agg = agg0;
        g.ld_agg = ld_agg;
        g.nb = nb;
        g.cap_rows = n_rows;  // (agg0 has n_rows rows; nb has cap_rows >= n_rows)
        g.gz = head ? head->g : nullptr;
        g.gz_ld = static_cast<int>(C4);
        g.gz_rows = head ? static_cast<int>(head->g_rows) : 0;
        g.gz_rows_dev = head ? head->g_rows_dev : nullptr;
        g.cnt_y = head ? head->y : nullptr;
        g.cnt_B = head ? static_cast<int>(head->B) : 0;
        g.cnt_ignore = head ? head->ignore_index : 0;
        g.cnt_out = head ? reinterpret_cast<float *>(static_cast<char *>(head->ws) + 4) : nullptr;
        g.scnt_base = (head && head->g) ? head->src_count : nullptr;
        g.scnt_stride = static_cast<int>(head ? head->g_rows : 0);
        const int tiles = static_cast<int>(ceil_div(g.n_edge, 16));
        const int grid = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(ncu, tiles)));
        int rc = NGNN_E_SHAPE;
#ifdef NGNN_FWD2_DBG_BUILD
        if (const char *d = getenv("NGNN_EDGE_DBG")) {
            switch (C0 == 4 ? atoi(d) : 0) {
                case 1: return launch_edge_nb<4, 1>(g, grid, st);
                case 2: return launch_edge_nb<4, 2>(g, grid, st);
                case 3: return launch_edge_nb<4, 3>(g, grid, st);
                case 4: return launch_edge_nb<4, 4>(g, grid, st);
                case 6: return launch_edge_nb<4, 6>(g, grid, st);
                case 7: return launch_edge_nb<4, 7>(g, grid, st);
                case 8: return launch_edge_nb<4, 8>(g, grid, st);
                case 16: return launch_edge_nb<4, 16>(g, grid, st);
                case 23: return launch_edge_nb<4, 23>(g, grid, st);
                case 24: return launch_edge_nb<4, 24>(g, grid, st);
                default: break;
            }
        }
#endif
        if (!fuse) {
            if (C0 == 4) rc = launch_edge_nb<4>(g, grid, st);
            if (rc) return rc;
        }
    } else if ((stages & NGNN_SAGE2_EDGE) && head && head->g && head->g_rows > 0) {
        // (no edge launch to zero the head's g: every row up to its static bound)
        const hipError_t e = hipMemsetAsync(head->g, 0, static_cast<size_t>(head->g_rows * C4 * 4), st);
        if (e != hipSuccess) return static_cast<int>(e);
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
        f.wr0 = wr0;
        f.ldw0 = ldw0;
        f.wr1 = wr1;
        f.wl1 = wl1;
        f.ldw1 = ldw1;
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
#ifdef NGNN_FWD2_DBG_BUILD
        if (const char *d = getenv("NGNN_FWD2_DBG")) {
            const int v = atoi(d);
            if (C0 == 4 && NT1 == 3 && dm == 2 && !indexed) {
                switch (v) {
                    case 1: return launch_fwd2<4, 3, 2, false, 1>(f, grid, st);
                    case 2: return launch_fwd2<4, 3, 2, false, 2>(f, grid, st);
                    case 3: return launch_fwd2<4, 3, 2, false, 3>(f, grid, st);
                    case 4: return launch_fwd2<4, 3, 2, false, 4>(f, grid, st);
                    case 8: return launch_fwd2<4, 3, 2, false, 8>(f, grid, st);
                    case 15: return launch_fwd2<4, 3, 2, false, 15>(f, grid, st);
                    case 16: return launch_fwd2<4, 3, 2, false, 16>(f, grid, st);
                    case 32: return launch_fwd2<4, 3, 2, false, 32>(f, grid, st);
                    case 64: return launch_fwd2<4, 3, 2, false, 64>(f, grid, st);
                    default: break;
                }
            }
        }
#endif
        // (K0 <= 112: the 16-deep tail chunk; NGNN_FWD2_T16=0 forces 4 x 32 -- A/B)
        static const bool t16_ok = [] {
            const char *v = std::getenv("NGNN_FWD2_T16");
            return !(v && v[0] == '0');
        }();
        const bool t16 = t16_ok && K0 <= 112;
        auto go = [&](auto xr_c) {
            constexpr bool XRv = decltype(xr_c)::value;
            if (!wr0) {  // (root-free: no x, so no T16 form; never indexed)
                if (fuse)
                    return dm == 2   ? launch_fwd2x<4, 3, 2, false, false, false>(g, f, grid, st)
                           : dm == 1 ? launch_fwd2x<4, 3, 1, false, false, false>(g, f, grid, st)
                                     : launch_fwd2x<4, 3, 0, false, false, false>(g, f, grid, st);
                return dm == 2   ? launch_fwd2<4, 3, 2, false, 0, false, false>(f, grid, st)
                       : dm == 1 ? launch_fwd2<4, 3, 1, false, 0, false, false>(f, grid, st)
                                 : launch_fwd2<4, 3, 0, false, 0, false, false>(f, grid, st);
            }
            if (fuse) {
                if (t16)
                    return dm == 2   ? launch_fwd2x<4, 3, 2, XRv, true>(g, f, grid, st)
                           : dm == 1 ? launch_fwd2x<4, 3, 1, XRv, true>(g, f, grid, st)
                                     : launch_fwd2x<4, 3, 0, XRv, true>(g, f, grid, st);
                return dm == 2   ? launch_fwd2x<4, 3, 2, XRv>(g, f, grid, st)
                       : dm == 1 ? launch_fwd2x<4, 3, 1, XRv>(g, f, grid, st)
                                 : launch_fwd2x<4, 3, 0, XRv>(g, f, grid, st);
            }
            if (t16)
                return dm == 2   ? launch_fwd2<4, 3, 2, XRv, 0, true>(f, grid, st)
                       : dm == 1 ? launch_fwd2<4, 3, 1, XRv, 0, true>(f, grid, st)
                                 : launch_fwd2<4, 3, 0, XRv, 0, true>(f, grid, st);
            return dm == 2   ? launch_fwd2<4, 3, 2, XRv>(f, grid, st)
                   : dm == 1 ? launch_fwd2<4, 3, 1, XRv>(f, grid, st)
                             : launch_fwd2<4, 3, 0, XRv>(f, grid, st);
        };
        if (C0 == 4 && NT1 == 3) rc = indexed ? go(std::true_type{}) : go(std::false_type{});
        if (rc) return rc;
    }
    if (!(stages & NGNN_SAGE2_NARROW)) return NGNN_OK;
    NarrowHead nh{};
    if (head) {
        nh.y = head->y;
        nh.B = static_cast<int>(head->B);
        nh.ignore = head->ignore_index;
        nh.loss = head->loss;
        nh.count = head->count;
        nh.dy = head->dy;
        nh.ldd = head->ldd;
        nh.g = head->g;
        nh.ldg = static_cast<int>(C4);
        nh.ticket = static_cast<uint32_t *>(head->ws);
        nh.part = reinterpret_cast<float *>(static_cast<char *>(head->ws) + 256);
        // the count from this call's edge launch (ws + 4), else counted there
        nh.cnt_in = ((stages & NGNN_SAGE2_EDGE) && n_edge_rows > 0)
                        ? reinterpret_cast<const float *>(static_cast<char *>(head->ws) + 4)
                        : nullptr;
        // the seed-edge counts only when this call's edge launch counted them
        if ((stages & NGNN_SAGE2_EDGE) && n_edge_rows > 0 && head->g) {
            nh.scnt_base = head->src_count;
            nh.scnt_stride = static_cast<int>(head->g_rows);
        }
#ifdef NGNN_FWD2_DBG_BUILD
        if (const char *d = getenv("NGNN_HEAD_DBG")) {
            nh.dbg = atoi(d);
            if (nh.dbg & 16) nh.cnt_in = reinterpret_cast<const float *>(static_cast<char *>(head->ws) + 4);
        }
#endif
    }
    return narrow_agg_launch(z, ldz, F1, rowptr, col, n_rows, n_rows_dev, n_edge_rows, n_edge_rows_dev, reduce,
                             out, ldo, st, head ? &nh : nullptr);
}
