// Wide SAGEConv layer forward for gfx950: layers whose weight image does not
// fit the row-tile kernel's LDS for more than two column slices -- Amazon-
// Computers' 767 -> 512 max layer (config_amazon.yml:11-14), where the
// row-tile kernel would re-read x in 16 slices and the 64-row kernel ran
// 128 workgroups on 256 CUs (460 us, 12 % of the f32 MFMA peak).
//
// Same contract as one SAGEConv layer of sage.py:33-39 (PyG 2.5.1
// SAGEConv.forward + relu + F.dropout):
//     out = act( b + x W_r^T + [deg > 0] agg(x) W_l^T )
// as TWO launches:
//   k_wide_agg   one wave per target row with in-edges: agg[d] = mean / sum /
//                max over its in-neighbours, walked in edge order (the fp32
//                sequence of ngnn_seg_agg_fwd: bit-identical aggregate), written
//                to the caller's saved-aggregate buffer (the backward's input);
//   k_wide_gemm  a 2-D tiled dual GEMM over [x | agg] . [W_r ; W_l]^T on exact
//                fp32 MFMA (v_mfma_f32_16x16x4_f32, like the 64-row kernel),
//                64 rows x 128 output columns per 256-thread workgroup, K staged
//                through double-buffered LDS 32 at a time (one barrier per
//                stage), the next stage's global loads in flight during the
//                current stage's MFMAs; tiles past the rows with in-edges skip
//                the W_l half.  Epilogue from the accumulators: bias, ReLU,
//                hash dropout (the same keys as every other forward kernel),
//                16-B stores (a lane holds 4 consecutive columns of one row).
//   Persistent workgroups over the LIVE tiles (device row count), tile t =
//   blockIdx + j gridDim with the grid a multiple of 8: each XCD (linear id %
//   8) keeps to fixed column tiles, so its L2 holds only its slice of W.
//
// Roofline: flops 2 N K F_out + 2 N_edge K F_out on the
// 157.3 TF f32 MFMA peak; bytes x (N K 4) + gathered rows (E K 4) + agg write
// and re-read (2 N_edge K 4) + out (N F_out 4).
#include <algorithm>
#include <cstdlib>

#include "ngnn_device.h"

namespace ngnn {
namespace {

constexpr int WBM = 64;        // rows per tile
constexpr int WBN = 128;       // output columns per tile
constexpr int WKC = 32;        // k per LDS stage
constexpr int WLD = WKC + 4;   // LDS row stride (floats): 16 rows hit 16 distinct 4-bank groups
constexpr int WSTAGE = (WBM + WBN) * WLD;  // floats per stage buffer
constexpr int WXU = WBM * WKC / 256;       // x / agg loads per thread per stage (8)
constexpr int WWU = WBN * WKC / 256;       // weight loads per thread per stage (16)

// ---- aggregate rows [0, min(n_rows, *n_rows_dev, *n_edge_dev)): one wave
// per row, lane owns columns p0 + lane + 64 c (c < NC); neighbour ids loaded
// 64 at a time and broadcast; two neighbour rows in flight, reduced in order.
// The H2 layer's preparation (k_wide_prep_h2, below) riding on the
// aggregate's launch: workgroups [n_agg, grid) split the W rows and take the
// x rows' exponents while [0, n_agg) aggregate -- the two are independent,
// and the preparation's x pass overlaps the gathers instead of following
// them as a launch of its own.  img == nullptr: no preparation.
struct WidePrep {
    const float *wr, *wl;
    int64_t ldw;
    int Fo, Kp;
    _Float16 *img;
    int *ew;
    int nbw;     // workgroups of W rows (4 rows each)
    int n_rows;  // x rows whose exponents are taken
    int *ex;
    int n_agg;   // the aggregate's workgroups
};
__device__ void wide_prep_body(const WidePrep &pp, const float *x, const float *const *x_dev, int64_t ldx, int K,
                               const int32_t *n_rows_dev, int bid, int nblk);

template <int RED, int NC>
__global__ __launch_bounds__(256) void k_wide_agg(const float *__restrict__ x, int64_t ldx, int K,
                                                  const int32_t *__restrict__ rowptr,
                                                  const int32_t *__restrict__ col, int n_rows,
                                                  const int32_t *__restrict__ n_rows_dev,
                                                  const int32_t *__restrict__ n_edge_dev,
                                                  float *__restrict__ agg, int64_t ld_agg,
                                                  int n_cap, int round16,
                                                  const float *const *x_dev, int *__restrict__ ea, WidePrep pp) {
    if (pp.img && static_cast<int>(blockIdx.x) >= pp.n_agg) {
        wide_prep_body(pp, x, x_dev, ldx, K, n_rows_dev, static_cast<int>(blockIdx.x) - pp.n_agg,
                       static_cast<int>(gridDim.x) - pp.n_agg);
        return;
    }
    const int n_blk = pp.img ? pp.n_agg : static_cast<int>(gridDim.x);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (x_dev) x = gload(x_dev, 0);  // (a graph slot's batch address, read at run time)
    int rows = n_rows;
    if (n_edge_dev) rows = min(rows, *n_edge_dev);
    // round16: rows up to the end of the last 16-row tile with in-edges (the
    // row-tile kernel reads the aggregate of whole tiles; those rows have no
    // in-edges and get 0)
    if (round16) rows = (rows + 15) & ~15;
    rows = min(rows, n_cap);
    if (n_rows_dev) rows = min(rows, *n_rows_dev);
    const float init = (RED == NGNN_REDUCE_MAX) ? -INFINITY : 0.0f;
    for (int64_t d = static_cast<int64_t>(blockIdx.x) * 4 + wave; d < rows; d += n_blk * 4) {
        const int beg = rowptr[d], end = rowptr[d + 1];
        float am = 0.0f;  // (ea: the row's |max| -> its H2 staging exponent)
        for (int p0 = 0; p0 < K; p0 += 64 * NC) {
            float acc[NC];
#pragma unroll
            for (int c = 0; c < NC; ++c) acc[c] = init;
            for (int eb = beg; eb < end; eb += 64) {
                const int n = min(64, end - eb);
                const int myc = lane < n ? col[eb + lane] : 0;
                int k = 0;
                for (; k + 2 <= n; k += 2) {
                    const int64_t j0 = __shfl(myc, k), j1 = __shfl(myc, k + 1);
                    float v0[NC], v1[NC];
#pragma unroll
                    for (int c = 0; c < NC; ++c) {
                        const int f = p0 + lane + 64 * c;
                        v0[c] = f < K ? x[j0 * ldx + f] : 0.0f;
                        v1[c] = f < K ? x[j1 * ldx + f] : 0.0f;
                    }
#pragma unroll
                    for (int c = 0; c < NC; ++c) {
                        if (RED == NGNN_REDUCE_MAX) {
                            acc[c] = nanmax(acc[c], v0[c]);
                            acc[c] = nanmax(acc[c], v1[c]);
                        } else {
                            acc[c] = acc[c] + v0[c];
                            acc[c] = acc[c] + v1[c];
                        }
                    }
                }
                if (k < n) {
                    const int64_t j0 = __shfl(myc, k);
#pragma unroll
                    for (int c = 0; c < NC; ++c) {
                        const int f = p0 + lane + 64 * c;
                        const float v = f < K ? x[j0 * ldx + f] : 0.0f;
                        acc[c] = (RED == NGNN_REDUCE_MAX) ? nanmax(acc[c], v) : acc[c] + v;
                    }
                }
            }
            const int deg = end - beg;
            const float cnt = static_cast<float>(deg > 1 ? deg : 1);
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const int f = p0 + lane + 64 * c;
                if (f >= K) continue;
                float v = acc[c];
                if (RED == NGNN_REDUCE_MEAN) v = v / cnt;
                if (RED == NGNN_REDUCE_MAX && deg == 0) v = 0.0f;
                agg[d * ld_agg + f] = v;
                am = fmaxf(am, fabsf(v));
            }
        }
        if (ea) {
            const int e = h2_exp(wave_max(am));
            if (lane == 0) ea[d] = e;
        }
    }
}

struct WideArgs {
    const float *x;
    const float *const *x_dev;  // non-null: x's address read at run time (a graph slot's batch, zero-copy)
    int64_t ldx;
    const float *agg;  // NULL: no neighbour term
    int64_t ld_agg;
    const float *wr;   // NULL: no root term (GCNConv's aggregate-first form)
    const float *wl;
    int64_t ldw;
    int K, Fo, n_rows, n_edge;
    const int32_t *n_rows_dev, *n_edge_dev;
    float *out;
    int64_t ldo;
    Epi epi;
    const uint64_t *seed_dev;
    int n_ct;  // column tiles
    int xcd;   // k_wide_h2: a row tile's column tiles on one XCD (grid a multiple of 8)
};

template <bool VOUT>
__global__ __launch_bounds__(256, 2) void k_wide_gemm(WideArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[2 * WSTAGE];
    if (a.x_dev) a.x = gload(a.x_dev, 0);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    int rows = a.n_rows;
    if (a.n_rows_dev) rows = min(rows, *a.n_rows_dev);
    int erows = min(a.n_edge, rows);
    if (a.n_edge_dev) erows = min(erows, *a.n_edge_dev);
    const int nK = (a.K + WKC - 1) / WKC;
    const int c_root = a.wr ? nK : 0;  // root stages
    // live tiles (device row count); tile t = row tile t / n_ct, column tile
    // t % n_ct.  Persistent workgroups take t = blockIdx.x + j gridDim.x; the
    // grid is a multiple of 8, so with n_ct | 8 every tile an XCD (linear id
    // % 8) runs has the same column tile(s): that XCD's L2 holds only its
    // slice of W, and the row tiles with in-edges (first in a NeighborLoader
    // block, twice the stages) spread over every workgroup.
    const int n_live = ((rows + WBM - 1) / WBM) * a.n_ct;

    float xr[WXU], wreg[WWU];
    // wave tile: 64 output columns (4 MFMA m-tiles) x 32 rows (2 n-tiles)
    const int wn = (wave & 1) * 64, wm = (wave >> 1) * 32;
    const int i16 = lane & 15, q = lane >> 4;
    Dropout drop = a.epi.drop;
    if (a.seed_dev) drop.reseed(*a.seed_dev);

    for (int t = blockIdx.x; t < n_live; t += gridDim.x) {
        const int rt = t / a.n_ct, ct = t - rt * a.n_ct;
        const int r0 = rt * WBM, n0 = ct * WBN;
        const int nch = c_root + ((a.agg && r0 < erows) ? nK : 0);  // + neighbour stages
        auto load = [&](int c) {
            const bool nb = c >= c_root;
            const int kc = (nb ? c - c_root : c) * WKC;
            const float *src = nb ? a.agg : a.x;
            const int64_t ld = nb ? a.ld_agg : a.ldx;
            const int rlim = nb ? erows : rows;
            const float *w = nb ? a.wl : a.wr;
#pragma unroll
            for (int u = 0; u < WXU; ++u) {
                const int idx = u * 256 + tid, r = idx >> 5, k = idx & 31;
                xr[u] = (r0 + r < rlim && kc + k < a.K) ? src[(r0 + r) * ld + kc + k] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < WWU; ++u) {
                const int idx = u * 256 + tid, n = idx >> 5, k = idx & 31;
                wreg[u] = (n0 + n < a.Fo && kc + k < a.K)
                              ? w[static_cast<int64_t>(n0 + n) * a.ldw + kc + k]
                              : 0.0f;
            }
        };
        auto store = [&](float *s) {
#pragma unroll
            for (int u = 0; u < WXU; ++u) {
                const int idx = u * 256 + tid;
                s[(idx >> 5) * WLD + (idx & 31)] = xr[u];
            }
#pragma unroll
            for (int u = 0; u < WWU; ++u) {
                const int idx = u * 256 + tid;
                s[(WBM + (idx >> 5)) * WLD + (idx & 31)] = wreg[u];
            }
        };
        v4f acc[4][2];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = v4f{0.f, 0.f, 0.f, 0.f};

        if (nch > 0) {
            load(0);
            store(lds);
            __syncthreads();
        }
        for (int c = 0; c < nch; ++c) {
            const bool more = c + 1 < nch;
            if (more) load(c + 1);  // in flight during this stage's MFMAs
            const float *s = lds + (c & 1) * WSTAGE;
            // k mapping inside a stage: lane group q takes k = 8 q + step, so
            // each operand is two ds_read_b128 per tile for all 8 steps
            v4f wa[4][2], xb[2][2];
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
                const float *p = s + (WBM + wn + mt * 16 + i16) * WLD + 8 * q;
                wa[mt][0] = *reinterpret_cast<const v4f *>(p);
                wa[mt][1] = *reinterpret_cast<const v4f *>(p + 4);
            }
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                const float *p = s + (wm + nt * 16 + i16) * WLD + 8 * q;
                xb[nt][0] = *reinterpret_cast<const v4f *>(p);
                xb[nt][1] = *reinterpret_cast<const v4f *>(p + 4);
            }
#pragma unroll
            for (int st = 0; st < 8; ++st)
#pragma unroll
                for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                    for (int nt = 0; nt < 2; ++nt)
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                            wa[mt][st >> 2][st & 3], xb[nt][st >> 2][st & 3], acc[mt][nt], 0, 0, 0);
            if (more) store(lds + ((c + 1) & 1) * WSTAGE);
            __syncthreads();
        }

        // ---- epilogue: lane holds columns n0 + wn + 16 mt + 4 q + (0..3) of
        // row r0 + wm + 16 nt + i16
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
            const int r = r0 + wm + nt * 16 + i16;
            if (r >= rows) continue;
            const uint32_t rk = drop.row_key(static_cast<uint32_t>(r));
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
                const int c0 = n0 + wn + mt * 16 + 4 * q;
                if (c0 >= a.Fo) continue;
                const uint32_t kb =
                    drop.thresh ? drop.keep4(rk, static_cast<uint32_t>(a.epi.col_base + c0) >> 2) : 0xfu;
                v4f v = acc[mt][nt];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float e = v[j];
                    if (a.epi.bias && c0 + j < a.Fo) e += a.epi.bias[c0 + j];
                    if (a.epi.relu) e = (e < 0.0f) ? 0.0f : e;  // NaN passes, like torch.relu
                    if (drop.thresh) e = ((kb >> j) & 1u) ? e * drop.scale : 0.0f;
                    v[j] = e;
                }
                float *o = a.out + static_cast<int64_t>(r) * a.ldo + c0;
                if (VOUT && c0 + 4 <= a.Fo) {
                    *reinterpret_cast<v4f *>(o) = v;
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (c0 + j < a.Fo) o[j] = v[j];
                }
            }
        }
    }
}

// ---- the split-bf16 (X3) form of k_wide_gemm: the same tiles, stages and
// epilogue, the products on v_mfma_f32_16x16x32_bf16.  Each operand value v =
// v1 + v2 + v3 (bf16, RNE; |v - v1 - v2 - v3| <= 2^-24 |v|) and the six
// products whose magnitude reaches 2^-18 of the leading one (v1w1, v1w2,
// v2w1, v2w2, v1w3, v3w1; each exact in fp32) -- the row-tile kernel's
// root-term arithmetic (ngnn_sage_rt.hip), here for the
// neighbour term too: 16 cycles per 32-deep k-step and product against 256
// for the exact f32 steps (2.7x fewer MFMA cycles).  W_r / W_l are split ONCE
// per launch into a global image (k_wide_wimg: [mat][part][Fo][Kp] bf16, Kp =
// K rounded up to 32, zero padded); x / agg are split when a stage is staged.
// LDS rows are 32 bf16 (one stage) in four 16-B chunks, chunk c of row r at
// position c ^ ((r >> 2) & 3): the fragment reads (16 rows x one chunk per
// 16 lanes) and the staging writes are bank-conflict free.
constexpr int XW_STAGE = 3 * WBM * WKC + 3 * WBN * WKC;  // bf16 per stage buffer (36 KiB)

__global__ __launch_bounds__(256) void k_wide_wimg(const float *__restrict__ wr, const float *__restrict__ wl,
                                                   int64_t ldw, int Fo, int K, int Kp,
                                                   __bf16 *__restrict__ img) {
    const int64_t per = static_cast<int64_t>(Fo) * Kp;  // bf16 per part
    const int64_t idx = (blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x) * 8;
    if (idx >= 2 * per) return;
    const int mat = static_cast<int>(idx / per);
    const int64_t e = idx - mat * per;
    const int n = static_cast<int>(e / Kp), k0 = static_cast<int>(e - static_cast<int64_t>(n) * Kp);
    const float *w = mat ? wl : wr;
    typedef __bf16 b8 __attribute__((ext_vector_type(8)));
    b8 p1, p2, p3;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float v = (w && k0 + j < K) ? w[static_cast<int64_t>(n) * ldw + k0 + j] : 0.0f;
        const __bf16 h1 = static_cast<__bf16>(v);
        const float r1 = v - static_cast<float>(h1);
        const __bf16 h2 = static_cast<__bf16>(r1);
        p1[j] = h1;
        p2[j] = h2;
        p3[j] = static_cast<__bf16>(r1 - static_cast<float>(h2));
    }
    __bf16 *o = img + static_cast<int64_t>(mat) * 3 * per + e;
    *reinterpret_cast<b8 *>(o) = p1;
    *reinterpret_cast<b8 *>(o + per) = p2;
    *reinterpret_cast<b8 *>(o + 2 * per) = p3;
}

template <bool VOUT>
__global__ __launch_bounds__(256, 2) void k_wide_x3(WideArgs a, const __bf16 *__restrict__ wimg, int Kp) {
    typedef __bf16 b8 __attribute__((ext_vector_type(8)));
    extern __shared__ __attribute__((aligned(16))) __bf16 xlds[];  // [2][XW_STAGE]
    if (a.x_dev) a.x = gload(a.x_dev, 0);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    int rows = a.n_rows;
    if (a.n_rows_dev) rows = min(rows, *a.n_rows_dev);
    int erows = min(a.n_edge, rows);
    if (a.n_edge_dev) erows = min(erows, *a.n_edge_dev);
    rows = __builtin_amdgcn_readfirstlane(rows);
    erows = __builtin_amdgcn_readfirstlane(erows);
    const int nK = (a.K + WKC - 1) / WKC;
    const int c_root = a.wr ? nK : 0;
    const int n_live = ((rows + WBM - 1) / WBM) * a.n_ct;
    const int64_t per = static_cast<int64_t>(a.Fo) * Kp;
    const int wn = (wave & 1) * 64, wm = (wave >> 1) * 32;
    const int i16 = lane & 15, q = lane >> 4;
    Dropout drop = a.epi.drop;
    if (a.seed_dev) drop.reseed(*a.seed_dev);
    // staging roles: x / agg row xr_r = tid >> 2, its 8 values of chunk tid & 3;
    // W row tid >> 1 (of 128), chunks 2 (tid & 1), + 1
    const int xr_r = tid >> 2, xr_c = tid & 3;
    const int w_n = tid >> 1, w_h = tid & 1;
    auto sw = [](int r, int c) { return c ^ ((r >> 2) & 3); };
    // x / agg rows through buffer resources (16-B loads at 4-B aligned
    // offsets; past the range: 0)
    const i32x4 xrs = make_rsrc_u(a.x, static_cast<uint32_t>(static_cast<int64_t>(rows) * a.ldx * 4));
    const i32x4 ars = make_rsrc_u(a.agg, static_cast<uint32_t>(a.agg ? static_cast<int64_t>(erows) * a.ld_agg * 4 : 0));
    // two register sets: stage c + 1 waits in one for its store while stage
    // c + 2's loads land in the other (the MFMA phase of a stage is ~0.8k
    // cycles here -- a one-stage prefetch left the load latency exposed)
    v4f xv[2][2];
    b8 wv[2][3][2];

    for (int t = blockIdx.x; t < n_live; t += gridDim.x) {
        const int rt = t / a.n_ct, ct = t - rt * a.n_ct;
        const int r0 = rt * WBM, n0 = ct * WBN;
        const int nch = c_root + ((a.agg && r0 < erows) ? nK : 0);
        auto load = [&](int c, v4f (&xd)[2], b8 (&wd)[3][2]) __attribute__((always_inline)) {
            const bool nb = c >= c_root;
            const int kc = (nb ? c - c_root : c) * WKC;
            const int r = r0 + xr_r;
            const int64_t ld = nb ? a.ld_agg : a.ldx;
            const int k = kc + 8 * xr_c;
            const int off = (r < (nb ? erows : rows) && k < a.K) ? static_cast<int>((r * ld + k) * 4) : static_cast<int>(0xF0000000u);
            const i32x4 rs = nb ? ars : xrs;
            if (off == static_cast<int>(0xF0000000u) || k + 8 <= a.K) {
                xd[0] = buf_load4(rs, off, 0, 0);
                xd[1] = buf_load4(rs, off == static_cast<int>(0xF0000000u) ? off : off + 16, 0, 0);
            } else {  // (the row's last values: element by element, nothing past K)
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    xd[j >> 2][j & 3] = buf_load1(rs, k + j < a.K ? off + 4 * j : static_cast<int>(0xF0000000u), 0, 0);
            }
            const int n = min(n0 + w_n, a.Fo - 1);
            const __bf16 *wb = wimg + (nb ? 3 * per : 0) + static_cast<int64_t>(n) * Kp + kc + 16 * w_h;
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                wd[p][0] = *reinterpret_cast<const b8 *>(wb + p * per);
                wd[p][1] = *reinterpret_cast<const b8 *>(wb + p * per + 8);
            }
        };
        auto store = [&](__bf16 *s, int c, const v4f (&xd)[2], const b8 (&wd)[3][2]) __attribute__((always_inline)) {
            const bool nb = c >= c_root;
            const int kq = a.K - ((nb ? c - c_root : c) * WKC + 8 * xr_c);  // valid values of the 8
            b8 p1, p2, p3;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float v = j < kq ? xd[j >> 2][j & 3] : 0.0f;  // (past K: the next row's values)
                const __bf16 h1 = static_cast<__bf16>(v);
                const float r1 = v - static_cast<float>(h1);
                const __bf16 h2 = static_cast<__bf16>(r1);
                p1[j] = h1;
                p2[j] = h2;
                p3[j] = static_cast<__bf16>(r1 - static_cast<float>(h2));
            }
            const int xo = xr_r * WKC + 8 * sw(xr_r, xr_c);
            *reinterpret_cast<b8 *>(s + xo) = p1;
            *reinterpret_cast<b8 *>(s + WBM * WKC + xo) = p2;
            *reinterpret_cast<b8 *>(s + 2 * WBM * WKC + xo) = p3;
            __bf16 *ws = s + 3 * WBM * WKC;
            const bool wok = n0 + w_n < a.Fo;  // (rows past F_out: zero)
#pragma unroll
            for (int p = 0; p < 3; ++p)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    *reinterpret_cast<b8 *>(ws + p * WBN * WKC + w_n * WKC + 8 * sw(w_n, 2 * w_h + h)) =
                        wok ? wd[p][h] : b8{};
        };
        v4f acc[4][2];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = v4f{0.f, 0.f, 0.f, 0.f};
        auto mfma_stage = [&](const __bf16 *s) __attribute__((always_inline)) {
            const __bf16 *ws = s + 3 * WBM * WKC;
            b8 xb[2][3];
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                const int r = wm + 16 * nt + i16;
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    xb[nt][p] = *reinterpret_cast<const b8 *>(s + p * WBM * WKC + r * WKC + 8 * sw(r, q));
            }
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
                const int n = wn + 16 * mt + i16;
                b8 w[3];
#pragma unroll
                for (int p = 0; p < 3; ++p) w[p] = *reinterpret_cast<const b8 *>(ws + p * WBN * WKC + n * WKC + 8 * sw(n, q));
#pragma unroll
                for (int nt = 0; nt < 2; ++nt) {
                    v4f t2 = acc[mt][nt];
                    t2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[2], xb[nt][0], t2, 0, 0, 0);
                    t2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], xb[nt][2], t2, 0, 0, 0);
                    t2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], xb[nt][1], t2, 0, 0, 0);
                    t2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1], xb[nt][0], t2, 0, 0, 0);
                    t2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], xb[nt][1], t2, 0, 0, 0);
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], xb[nt][0], t2, 0, 0, 0);
                }
            }
        };
        if (nch > 0) {
            load(0, xv[0], wv[0]);
            if (nch > 1) load(1, xv[1], wv[1]);
            store(xlds, 0, xv[0], wv[0]);
            __syncthreads();
        }
        // stage c: MFMAs from LDS[c & 1]; stage c + 1's registers (set (c+1) & 1)
        // go to LDS[(c+1) & 1] after them; stage c + 2 loads into set c & 1
        // (compile-time set indices: the loop runs in pairs)
        auto one = [&](int c, auto u_c) __attribute__((always_inline)) {
            constexpr int U = decltype(u_c)::value;  // c & 1
            if (c + 2 < nch) load(c + 2, xv[U], wv[U]);
            mfma_stage(xlds + U * XW_STAGE);
            if (c + 1 < nch) store(xlds + (U ^ 1) * XW_STAGE, c + 1, xv[U ^ 1], wv[U ^ 1]);
            __syncthreads();
        };
        for (int c = 0; c < nch; c += 2) {
            one(c, std::integral_constant<int, 0>{});
            if (c + 1 < nch) one(c + 1, std::integral_constant<int, 1>{});
        }
        // ---- epilogue (k_wide_gemm's): lane holds columns n0 + wn + 16 mt +
        // 4 q + (0..3) of row r0 + wm + 16 nt + i16
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
            const int r = r0 + wm + nt * 16 + i16;
            if (r >= rows) continue;
            const uint32_t rk = drop.row_key(static_cast<uint32_t>(r));
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
                const int c0 = n0 + wn + mt * 16 + 4 * q;
                if (c0 >= a.Fo) continue;
                const uint32_t kb =
                    drop.thresh ? drop.keep4(rk, static_cast<uint32_t>(a.epi.col_base + c0) >> 2) : 0xfu;
                v4f v = acc[mt][nt];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float e = v[j];
                    if (a.epi.bias && c0 + j < a.Fo) e += a.epi.bias[c0 + j];
                    if (a.epi.relu) e = (e < 0.0f) ? 0.0f : e;  // NaN passes, like torch.relu
                    if (drop.thresh) e = ((kb >> j) & 1u) ? e * drop.scale : 0.0f;
                    v[j] = e;
                }
                float *o = a.out + static_cast<int64_t>(r) * a.ldo + c0;
                if (VOUT && c0 + 4 <= a.Fo) {
                    *reinterpret_cast<v4f *>(o) = v;
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (c0 + j < a.Fo) o[j] = v[j];
                }
            }
        }
    }
}

// ---- the H2 form (round 5): two fp16 parts per operand after a
// power-of-two scaling -- each x / agg row by its own max, each W row (an
// output column) by its own -- and THREE v_mfma_f32_16x16x32_f16 products
// per k-step (w1 x2, w2 x1, w1 x1; each exact in fp32: ~3 2^-22 relative,
// the two-layer kernels' arithmetic) instead of X3's
// six bf16 ones; the weight image is 2 parts instead of 3.  The scales must
// be known before a row's first k-stage, so the row exponents come from a
// pass (k_wide_prep_h2, with the W split and the W rows' exponents), the
// aggregate rows' from k_wide_agg as it stores them; the
// root and neighbour terms have different row and column scales, so they
// accumulate apart and meet, unscaled, in the epilogue.
// halves per stage buffer (BM = 64: 24 KiB); BM = 128 (eight waves): the W
// tile staged once per 128 rows -- half the image's L2 reads per row
template <int BM>
constexpr int hw_stage() { return 2 * BM * WKC + 2 * WBN * WKC; }
typedef _Float16 h8w __attribute__((ext_vector_type(8)));

// one wave per W row (mat, n): its exponent (max |w| of the row in [2^14,
// 2^15) after scaling) and its two fp16 parts -> img [mat][part][Fo][Kp]
__device__ __forceinline__ void wimg_h2_row(const float *__restrict__ wr, const float *__restrict__ wl, int64_t ldw,
                                            int Fo, int K, int Kp, _Float16 *__restrict__ img, int *__restrict__ ew,
                                            int row, int lane) {
    const int mat = row / Fo, n = row - mat * Fo;
    const float *w = mat ? wl : wr;
    // (8 consecutive values per lane and pass, 16-B part stores; the second
    // pass re-reads the row from L2)
    const float *wrow = w ? w + static_cast<int64_t>(n) * ldw : nullptr;
    auto get8 = [&](int k0, float (&v)[8]) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (wrow && k0 + j < K) ? wrow[k0 + j] : 0.0f;
    };
    float m = 0.0f;
    for (int kb = 0; kb < Kp; kb += 512) {
        float v[8];
        get8(kb + 8 * lane, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[j]));
    }
    const int e = h2_exp(wave_max(m));
    if (lane == 0) ew[row] = e;
    const int64_t per = static_cast<int64_t>(Fo) * Kp;
    _Float16 *o = img + static_cast<int64_t>(2 * mat) * per + static_cast<int64_t>(n) * Kp;
    for (int kb = 0; kb < Kp; kb += 512) {
        const int k0 = kb + 8 * lane;
        if (k0 >= Kp) break;  // (Kp is a multiple of 32: whole 8-blocks)
        float v[8];
        get8(k0, v);
        h8w p1, p2;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float s = __builtin_amdgcn_ldexpf(v[j], e);
            const _Float16 h = static_cast<_Float16>(s);
            p1[j] = h;
            p2[j] = static_cast<_Float16>(s - static_cast<float>(h));
        }
        *reinterpret_cast<h8w *>(o + k0) = p1;
        *reinterpret_cast<h8w *>(o + per + k0) = p2;
    }
}

// the H2 layer's preparation in one launch: workgroups [0, nbw) split the W
// rows (wimg_h2_row), the rest take one wave per x row [0, rows) -> ex (the
// root staging's exponents; the aggregate rows' come from k_wide_agg)
// (workgroup bid of nblk: the body shared with k_wide_agg's riders)
__device__ void wide_prep_body(const WidePrep &pp, const float *x, const float *const *x_dev, int64_t ldx, int K,
                               const int32_t *n_rows_dev, int bid, int nblk) {
    const int lane = threadIdx.x & 63;
    if (bid < pp.nbw) {
        const int row = bid * 4 + (threadIdx.x >> 6);
        if (row < 2 * pp.Fo) wimg_h2_row(pp.wr, pp.wl, pp.ldw, pp.Fo, K, pp.Kp, pp.img, pp.ew, row, lane);
        return;
    }
    if (x_dev) x = gload(x_dev, 0);
    int rows = pp.n_rows;
    if (n_rows_dev) rows = min(rows, *n_rows_dev);
    const int waves = (nblk - pp.nbw) * 4;
    for (int r = (bid - pp.nbw) * 4 + (threadIdx.x >> 6); r < rows; r += waves) {
        const float *p = x + static_cast<int64_t>(r) * ldx;
        float m = 0.0f;
        for (int k = lane; k < K; k += 64) m = fmaxf(m, fabsf(p[k]));
        const int e = h2_exp(wave_max(m));
        if (lane == 0) pp.ex[r] = e;
    }
}

__global__ __launch_bounds__(256) void k_wide_prep_h2(WidePrep pp, const float *__restrict__ x,
                                                      const float *const *x_dev, int64_t ldx, int K,
                                                      const int32_t *__restrict__ n_rows_dev) {
    wide_prep_body(pp, x, x_dev, ldx, K, n_rows_dev, static_cast<int>(blockIdx.x), static_cast<int>(gridDim.x));
}

template <bool VOUT, int BM>
__global__ __launch_bounds__(BM * 4, 128 / BM) void k_wide_h2(WideArgs a, const _Float16 *__restrict__ wimg, int Kp,
                                                    const int *__restrict__ ew, const int *__restrict__ ex,
                                                    const int *__restrict__ ea) {
    constexpr int NTH = BM * 4;
    constexpr int STG = hw_stage<BM>();
    constexpr int PW = WBN * 4 / NTH;  // 8-half W pieces per thread and part (of a column's 4)
    extern __shared__ __attribute__((aligned(16))) _Float16 hlds[];  // [2][STG]
    if (a.x_dev) a.x = gload(a.x_dev, 0);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    int rows = a.n_rows;
    if (a.n_rows_dev) rows = min(rows, *a.n_rows_dev);
    int erows = min(a.n_edge, rows);
    if (a.n_edge_dev) erows = min(erows, *a.n_edge_dev);
    rows = __builtin_amdgcn_readfirstlane(rows);
    erows = __builtin_amdgcn_readfirstlane(erows);
    const int nK = (a.K + WKC - 1) / WKC;
    const int c_root = a.wr ? nK : 0;
    const int n_live = ((rows + BM - 1) / BM) * a.n_ct;
    const int64_t per = static_cast<int64_t>(a.Fo) * Kp;
    const int wn = (wave & 1) * 64, wm = (wave >> 1) * 32;
    const int i16 = lane & 15, q = lane >> 4;
    Dropout drop = a.epi.drop;
    if (a.seed_dev) drop.reseed(*a.seed_dev);
    const int xr_r = tid >> 2, xr_c = tid & 3;
    const int w_n = tid / (4 / PW), w_h = (tid % (4 / PW)) * PW;  // (column, first piece)
    auto sw = [](int r, int c) { return c ^ ((r >> 2) & 3); };
    const i32x4 xrs = make_rsrc_u(a.x, static_cast<uint32_t>(static_cast<int64_t>(rows) * a.ldx * 4));
    const i32x4 ars = make_rsrc_u(a.agg, static_cast<uint32_t>(a.agg ? static_cast<int64_t>(erows) * a.ld_agg * 4 : 0));
    v4f xv[2][2];
    h8w wv[2][2][PW];

    // XCD-aware order (workgroup b runs on XCD b mod 8): row tile rt goes to
    // XCD rt mod 8 with all its column tiles, so its x / agg rows are fetched
    // into one L2 instead of n_ct of them
    const int RT = (rows + BM - 1) / BM;
    const int xc = blockIdx.x & 7;
    const int n_mine = a.xcd ? (xc < RT ? (RT - xc + 7) / 8 : 0) * a.n_ct : n_live;
    const int t0 = a.xcd ? static_cast<int>(blockIdx.x >> 3) : static_cast<int>(blockIdx.x);
    const int ts = a.xcd ? static_cast<int>(gridDim.x >> 3) : static_cast<int>(gridDim.x);
    for (int u = t0; u < n_mine; u += ts) {
        const int um = u / a.n_ct, ct = u - um * a.n_ct;
        const int rt = a.xcd ? xc + 8 * um : um;
        const int r0 = rt * BM, n0 = ct * WBN;
        const int nch = c_root + ((a.agg && r0 < erows) ? nK : 0);
        // the staging row's scales (rows past the range: never stored)
        const int sr = r0 + xr_r;
        const int e_x = sr < rows ? ex[sr] : 0;
        const int e_a = (a.agg && sr < erows) ? ea[sr] : 0;
        auto load = [&](int c, v4f (&xd)[2], h8w (&wd)[2][PW]) __attribute__((always_inline)) {
            const bool nb = c >= c_root;
            const int kc = (nb ? c - c_root : c) * WKC;
            const int r = r0 + xr_r;
            const int64_t ld = nb ? a.ld_agg : a.ldx;
            const int k = kc + 8 * xr_c;
            const int off = (r < (nb ? erows : rows) && k < a.K) ? static_cast<int>((r * ld + k) * 4) : static_cast<int>(0xF0000000u);
            const i32x4 rs = nb ? ars : xrs;
            if (off == static_cast<int>(0xF0000000u) || k + 8 <= a.K) {
                xd[0] = buf_load4(rs, off, 0, 0);
                xd[1] = buf_load4(rs, off == static_cast<int>(0xF0000000u) ? off : off + 16, 0, 0);
            } else {  // (the row's last values: element by element, nothing past K)
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    xd[j >> 2][j & 3] = buf_load1(rs, k + j < a.K ? off + 4 * j : static_cast<int>(0xF0000000u), 0, 0);
            }
            const int n = min(n0 + w_n, a.Fo - 1);
            const _Float16 *wb = wimg + (nb ? 2 * per : 0) + static_cast<int64_t>(n) * Kp + kc + 8 * w_h;
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int h = 0; h < PW; ++h) wd[p][h] = *reinterpret_cast<const h8w *>(wb + p * per + 8 * h);
        };
        auto store = [&](_Float16 *s, int c, const v4f (&xd)[2], const h8w (&wd)[2][PW]) __attribute__((always_inline)) {
            const bool nb = c >= c_root;
            const int kq = a.K - ((nb ? c - c_root : c) * WKC + 8 * xr_c);  // valid values of the 8
            const int e = nb ? e_a : e_x;
            h8w p1, p2;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float v = j < kq ? __builtin_amdgcn_ldexpf(xd[j >> 2][j & 3], e) : 0.0f;  // (past K: 0)
                const _Float16 h = static_cast<_Float16>(v);
                p1[j] = h;
                p2[j] = static_cast<_Float16>(v - static_cast<float>(h));
            }
            const int xo = xr_r * WKC + 8 * sw(xr_r, xr_c);
            *reinterpret_cast<h8w *>(s + xo) = p1;
            *reinterpret_cast<h8w *>(s + BM * WKC + xo) = p2;
            _Float16 *ws = s + 2 * BM * WKC;
            const bool wok = n0 + w_n < a.Fo;  // (rows past F_out: zero)
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int h = 0; h < PW; ++h)
                    *reinterpret_cast<h8w *>(ws + p * WBN * WKC + w_n * WKC + 8 * sw(w_n, w_h + h)) =
                        wok ? wd[p][h] : h8w{};
        };
        v4f accr[4][2], accn[4][2];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) accr[mt][nt] = accn[mt][nt] = v4f{0.f, 0.f, 0.f, 0.f};
        auto mfma_stage = [&](const _Float16 *s, v4f (&acc)[4][2]) __attribute__((always_inline)) {
            const _Float16 *ws = s + 2 * BM * WKC;
            h8w xb[2][2];
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                const int r = wm + 16 * nt + i16;
#pragma unroll
                for (int p = 0; p < 2; ++p)
                    xb[nt][p] = *reinterpret_cast<const h8w *>(s + p * BM * WKC + r * WKC + 8 * sw(r, q));
            }
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
                const int n = wn + 16 * mt + i16;
                h8w w[2];
#pragma unroll
                for (int p = 0; p < 2; ++p) w[p] = *reinterpret_cast<const h8w *>(ws + p * WBN * WKC + n * WKC + 8 * sw(n, q));
#pragma unroll
                for (int nt = 0; nt < 2; ++nt) {
                    v4f t2 = acc[mt][nt];
                    t2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(w[0], xb[nt][1], t2, 0, 0, 0);
                    t2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(w[1], xb[nt][0], t2, 0, 0, 0);
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w[0], xb[nt][0], t2, 0, 0, 0);
                }
            }
        };
        if (nch > 0) {
            load(0, xv[0], wv[0]);
            if (nch > 1) load(1, xv[1], wv[1]);
            store(hlds, 0, xv[0], wv[0]);
            __syncthreads();
        }
        // stage c: MFMAs from LDS[c & 1] into the root or the neighbour
        // accumulators (compile-time: the two loops); the staging as X3's
        auto one = [&](int c, auto u_c, auto nb_c) __attribute__((always_inline)) {
            constexpr int U = decltype(u_c)::value;  // c & 1
            if (c + 2 < nch) load(c + 2, xv[U], wv[U]);
            if constexpr (decltype(nb_c)::value) mfma_stage(hlds + U * STG, accn);
            else mfma_stage(hlds + U * STG, accr);
            if (c + 1 < nch) store(hlds + (U ^ 1) * STG, c + 1, xv[U ^ 1], wv[U ^ 1]);
            __syncthreads();
        };
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        // (c_root is even: the host takes this form only for an even number
        // of k-stages, so both loops start on buffer 0)
        for (int c = 0; c < c_root; c += 2) {
            one(c, I0{}, std::false_type{});
            one(c + 1, I1{}, std::false_type{});
        }
        for (int c = c_root; c < nch; c += 2) {
            one(c, I0{}, std::true_type{});
            if (c + 1 < nch) one(c + 1, I1{}, std::true_type{});
        }
        // ---- epilogue: lane holds columns n0 + wn + 16 mt + 4 q + (0..3) of
        // row r0 + wm + 16 nt + i16; each term unscaled by its row's and its
        // column's exponents (exact), summed, then bias / ReLU / dropout
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
            const int r = r0 + wm + nt * 16 + i16;
            if (r >= rows) continue;
            const int erx = ex[r];
            const bool hn = a.agg && r < erows;
            const int era = hn ? ea[r] : 0;
            const uint32_t rk = drop.row_key(static_cast<uint32_t>(r));
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
                const int c0 = n0 + wn + mt * 16 + 4 * q;
                if (c0 >= a.Fo) continue;
                const uint32_t kb =
                    drop.thresh ? drop.keep4(rk, static_cast<uint32_t>(a.epi.col_base + c0) >> 2) : 0xfu;
                v4f v;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int cj = min(c0 + j, a.Fo - 1);
                    float e = __builtin_amdgcn_ldexpf(accr[mt][nt][j], -(erx + ew[cj]));
                    if (hn) e += __builtin_amdgcn_ldexpf(accn[mt][nt][j], -(era + ew[a.Fo + cj]));
                    if (a.epi.bias && c0 + j < a.Fo) e += a.epi.bias[c0 + j];
                    if (a.epi.relu) e = (e < 0.0f) ? 0.0f : e;  // NaN passes, like torch.relu
                    if (drop.thresh) e = ((kb >> j) & 1u) ? e * drop.scale : 0.0f;
                    v[j] = e;
                }
                float *o = a.out + static_cast<int64_t>(r) * a.ldo + c0;
                if (VOUT && c0 + 4 <= a.Fo) {
                    *reinterpret_cast<v4f *>(o) = v;
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (c0 + j < a.Fo) o[j] = v[j];
                }
            }
        }
    }
}

}  // namespace

// bytes of the wide layer's split weight image (k_wide_wimg)
size_t wide_wimg_bytes(int64_t K, int64_t Fo) {
    return static_cast<size_t>(2 * 3) * static_cast<size_t>(Fo) * static_cast<size_t>(ceil_div(K, 32) * 32) * 2;
}

// The row-tile kernel holds the W_r image of its whole column slice in LDS
// and re-reads x once per slice: the wide path takes a layer when F_out needs
// more than four such slices (or none fits), or K is not a multiple of 4 (the
// row-tile kernel reads 16-B column quads; the caller pads K when that keeps
// it within two slices, fused.pad_k_ok).  Its f32 MFMA rate is 1/2.7 of the
// row-tile kernel's split-bf16 root term, so moderately sliced layers (the
// 256 -> 256 hidden layer: 3 slices) stay on the row-tile kernel.
bool sage_wide_preferred(int64_t K, int64_t Fo, bool exact) {
    if (K % 4 != 0) return true;
    const int64_t KG = ceil_div(K, 16);
    int64_t C = K / 32, T4 = ceil_div(K % 32, 4);
    if (T4 > 3) {  // X3_TAIL_MAX (ngnn_sage_rt.hip): the tail becomes a padded chunk
        C += 1;
        T4 = 0;
    }
    const int64_t img = exact ? KG * 64 * 16 : 3 * C * 64 * 16 + T4 * 64 * 4;
    const int64_t cap = 160 * 1024 - 1024 - 256;
    int ntw = 0;
    for (int c : {16, 8, 6, 4, 3, 2})
        if (c * img <= cap) {
            ntw = c;
            break;
        }
    return ntw == 0 || ceil_div(Fo, 16 * ntw) > 4;
}

size_t sage_wide_workspace_bytes(int64_t K, int64_t n_rows) {
    return static_cast<size_t>(std::max<int64_t>(n_rows, 0)) * static_cast<size_t>(K) * sizeof(float);
}

int sage_fwd_wide(const float *x, int64_t ldx, int64_t K, int64_t n_rows,
                  const int32_t *n_rows_dev, int64_t n_edge_rows, const int32_t *n_edge_rows_dev,
                  const int32_t *rowptr, const int32_t *col, int reduce, const float *wl,
                  const float *wr, int64_t ldw, const float *bias, int64_t Fo, float *out,
                  int64_t ldo, int relu, float p_drop, uint64_t seed, const uint64_t *seed_dev,
                  float *agg_out, int64_t ld_agg, void *ws, size_t ws_bytes, hipStream_t st, bool exact,
                  const float *const *x_dev) {
    const int64_t n_edge = std::max<int64_t>(0, std::min(n_edge_rows, n_rows));
    // the H2 form (NGNN_WIDE_H2=0, read once: X3 -- A/B): an even number of
    // k-stages (its root / neighbour loops each start on buffer 0), 32-bit row
    // offsets, and room for the 2-part image + the row / column exponents at
    // the workspace tail -- decided first: the aggregation writes the
    // neighbour rows' exponents
    static const bool h2_on = [] {
        const char *e = std::getenv("NGNN_WIDE_H2");
        return !(e && e[0] == '0');
    }();
    const bool has_agg = wl && n_edge > 0;
    const int64_t lda_eff = agg_out ? ld_agg : K;
    const bool fits = n_rows * ldx * 4 < 0x7FFF0000ll && (!has_agg || n_edge * lda_eff * 4 < 0x7FFF0000ll);
    const size_t head = has_agg && (!agg_out || agg_out == ws) ? sage_wide_workspace_bytes(K, n_edge) : 0;
    const int Kp = static_cast<int>(ceil_div(K, 32) * 32);
    const size_t ib2 = static_cast<size_t>(4) * Fo * Kp * 2;
    const size_t side = (static_cast<size_t>(2) * Fo + n_rows + n_edge) * 4 + 1024;
    const bool use_h2 = !exact && h2_on && fits && ceil_div(K, WKC) % 2 == 0 && ws && ws_bytes >= head + ib2 + side + 512;
    _Float16 *h2_img = nullptr;
    int *ew = nullptr, *ex = nullptr, *ea = nullptr;
    if (use_h2) {
        const uintptr_t e = (reinterpret_cast<uintptr_t>(ws) + ws_bytes - ib2) & ~uintptr_t(255);
        h2_img = reinterpret_cast<_Float16 *>(e);
        ew = reinterpret_cast<int *>((e - side) & ~uintptr_t(255));
        ex = ew + 2 * Fo;
        ea = ex + n_rows;
    }
    int *const agg_ea = ea;
    // the preparation's workgroups: 4 W rows each, then one wave per x row
    // (capped); riding on the aggregate's launch when there is one
    WidePrep prep{};
    unsigned prep_blocks = 0;
    if (use_h2) {
        prep = WidePrep{wr, wl, ldw, static_cast<int>(Fo), Kp, h2_img, ew, static_cast<int>(ceil_div(2 * Fo, 4)),
                        static_cast<int>(n_rows), ex, 0};
        const int64_t gr = std::max<int64_t>(1, std::min<int64_t>(ceil_div(n_rows, 4), 8 * num_cus()));
        prep_blocks = static_cast<unsigned>(prep.nbw + gr);
    }
    bool prep_done = false;
    float *agg = nullptr;
    int64_t lda = ld_agg;
    if (has_agg) {
        if (agg_out) {
            agg = agg_out;
        } else {
            NGNN_RETURN_IF(!ws || ws_bytes < sage_wide_workspace_bytes(K, n_edge) || !aligned(ws, 4),
                           NGNN_E_WORKSPACE);
            agg = static_cast<float *>(ws);
            lda = K;
        }
        const unsigned ga = static_cast<unsigned>(std::min<int64_t>(ceil_div(n_edge, 4), 8 * num_cus()));
        prep.n_agg = static_cast<int>(ga);
        prep_done = use_h2;
        auto launch_agg = [&](auto red_c, auto nc_c) {
            hipLaunchKernelGGL((k_wide_agg<decltype(red_c)::value, decltype(nc_c)::value>), dim3(ga + prep_blocks),
                               dim3(256), 0, st, x, ldx, static_cast<int>(K), rowptr, col,
                               static_cast<int>(n_edge), n_rows_dev, n_edge_rows_dev, agg, lda,
                               static_cast<int>(n_rows), 0, x_dev, agg_ea, prep);
        };
        auto by_nc = [&](auto red_c) {
            if (K <= 256) launch_agg(red_c, std::integral_constant<int, 4>{});
            else if (K <= 512) launch_agg(red_c, std::integral_constant<int, 8>{});
            else launch_agg(red_c, std::integral_constant<int, 12>{});  // (> 768: passes of 768)
        };
        if (reduce == NGNN_REDUCE_MEAN) by_nc(std::integral_constant<int, NGNN_REDUCE_MEAN>{});
        else if (reduce == NGNN_REDUCE_SUM) by_nc(std::integral_constant<int, NGNN_REDUCE_SUM>{});
        else by_nc(std::integral_constant<int, NGNN_REDUCE_MAX>{});
        const int rc = launch_status();
        if (rc) return rc;
    }
    WideArgs a;
    a.x = x;
    a.x_dev = x_dev;
    a.ldx = ldx;
    a.agg = agg;
    a.ld_agg = lda;
    a.wr = wr;
    a.wl = wl;
    a.ldw = ldw;
    a.K = static_cast<int>(K);
    a.Fo = static_cast<int>(Fo);
    a.n_rows = static_cast<int>(n_rows);
    a.n_edge = static_cast<int>(n_edge);
    a.n_rows_dev = n_rows_dev;
    a.n_edge_dev = n_edge_rows_dev;
    a.out = out;
    a.ldo = ldo;
    a.epi = Epi{bias, relu, make_dropout(p_drop, seed), 0};
    a.seed_dev = seed_dev;
    a.n_ct = static_cast<int>(ceil_div(Fo, WBN));
    // (NGNN_WIDE_XCD=0, read once: k_wide_h2's plain tile order -- A/B)
    static const bool xcd_on = [] {
        const char *e = std::getenv("NGNN_WIDE_XCD");
        return !(e && e[0] == '0');
    }();
    a.xcd = 0;
    const int64_t tiles = ceil_div(n_rows, WBM) * a.n_ct;
    NGNN_RETURN_IF(tiles > INT32_MAX, NGNN_E_RANGE);
    // persistent: two workgroups per CU (55 KiB LDS, 178 VGPRs each), a
    // multiple of 8 (one per XCD in turn)
    const int64_t grid = std::max<int64_t>(8, std::min<int64_t>(ceil_div(tiles, 8) * 8, 2 * num_cus()));
    const bool vout = (ldo % 4 == 0) && aligned(out, 16);
    // the split-bf16 form (not under NGNN_MATH_EXACT_F32): its weight image at
    // the workspace's tail (NGNN_WIDE_X3=0, read once: the exact f32 form -- A/B)
    static const bool x3_on = [] {
        const char *e = std::getenv("NGNN_WIDE_X3");
        return !(e && e[0] == '0');
    }();
    const size_t ib = wide_wimg_bytes(K, Fo);
    {
        if (use_h2) {
            _Float16 *img = h2_img;
            if (!prep_done) {
                hipLaunchKernelGGL(k_wide_prep_h2, dim3(prep_blocks), dim3(256), 0, st, prep, x, x_dev, ldx,
                                   static_cast<int>(K), n_rows_dev);
                const int rc = launch_status();
                if (rc) return rc;
            }
            // (NGNN_WIDE_BM=128, read once: the eight-wave 128-row tile -- A/B)
            static const int bm = [] {
                const char *e = std::getenv("NGNN_WIDE_BM");
                return (e && std::atoi(e) == 128) ? 128 : 64;
            }();
            static bool attr_set[2][2] = {};
            auto go = [&](auto kern, int bm_c) {
                const size_t lds = static_cast<size_t>(2) * (2 * bm_c * WKC + 2 * WBN * WKC) * 2;
                bool &set = attr_set[vout][bm_c == 128];
                if (!set) {
                    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                                             static_cast<int>(lds));
                    if (e != hipSuccess) return static_cast<int>(e);
                    set = true;
                }
                const int64_t t2 = ceil_div(n_rows, bm_c) * a.n_ct;
                const int64_t g2 = std::max<int64_t>(8, std::min<int64_t>(ceil_div(t2, 8) * 8, (128 / bm_c) * num_cus()));
                a.xcd = (xcd_on && g2 % 8 == 0) ? 1 : 0;  // (the XCD order needs whole groups of 8)
                hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(g2)), dim3(bm_c * 4), lds, st, a, img, Kp, ew, ex, ea);
                return launch_status();
            };
            if (bm == 128) return vout ? go(k_wide_h2<true, 128>, 128) : go(k_wide_h2<false, 128>, 128);
            return vout ? go(k_wide_h2<true, 64>, 64) : go(k_wide_h2<false, 64>, 64);
        }
    }
    if (!exact && x3_on && fits && ws && ws_bytes >= head + ib + 256) {
        const uintptr_t e = (reinterpret_cast<uintptr_t>(ws) + ws_bytes - ib) & ~uintptr_t(255);
        __bf16 *img = reinterpret_cast<__bf16 *>(e);
        const int64_t nthr = static_cast<int64_t>(2) * Fo * Kp / 8;
        hipLaunchKernelGGL(k_wide_wimg, dim3(static_cast<unsigned>(ceil_div(nthr, 256))), dim3(256), 0, st, wr, wl,
                           ldw, static_cast<int>(Fo), static_cast<int>(K), Kp, img);
        int rc = launch_status();
        if (rc) return rc;
        const size_t lds = static_cast<size_t>(2) * XW_STAGE * 2;
        auto go = [&](auto v_c) {
            auto fn = k_wide_x3<decltype(v_c)::value>;
            static bool attr = false;  // benign race: idempotent
            if (!attr) {
                (void)hipFuncSetAttribute(reinterpret_cast<const void *>(fn),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
                attr = true;
            }
            hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(grid)), dim3(256), lds, st, a, img, Kp);
        };
        if (vout) go(std::true_type{});
        else go(std::false_type{});
        return launch_status();
    }
    if (vout)
        hipLaunchKernelGGL(k_wide_gemm<true>, dim3(static_cast<unsigned>(grid)), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL(k_wide_gemm<false>, dim3(static_cast<unsigned>(grid)), dim3(256), 0, st, a);
    return launch_status();
}

}  // namespace ngnn

namespace ngnn {
// The aggregate of rows [0, ceil16(min(n_edge_rows, *n_edge_rows_dev))) into
// agg (ld_agg), for the row-tile kernel's pre-aggregated max layers.
int sage_wide_aggregate(const float *x, int64_t ldx, int64_t K, int64_t n_rows,
                        const int32_t *n_rows_dev, int64_t n_edge_rows,
                        const int32_t *n_edge_rows_dev, const int32_t *rowptr, const int32_t *col,
                        int reduce, float *agg, int64_t ld_agg, hipStream_t st,
                        const float *const *x_dev) {
    const int64_t n_edge = std::max<int64_t>(0, std::min(ceil_div(n_edge_rows, 16) * 16, n_rows));
    if (n_edge == 0) return NGNN_OK;
    const unsigned ga = static_cast<unsigned>(std::min<int64_t>(ceil_div(n_edge, 4), 8 * num_cus()));
    auto launch_agg = [&](auto red_c, auto nc_c) {
        hipLaunchKernelGGL((k_wide_agg<decltype(red_c)::value, decltype(nc_c)::value>), dim3(ga),
                           dim3(256), 0, st, x, ldx, static_cast<int>(K), rowptr, col,
                           static_cast<int>(n_edge), n_rows_dev, n_edge_rows_dev, agg, ld_agg,
                           static_cast<int>(n_rows), 1, x_dev, nullptr, WidePrep{});
    };
    auto by_nc = [&](auto red_c) {
        if (K <= 256) launch_agg(red_c, std::integral_constant<int, 4>{});
        else if (K <= 512) launch_agg(red_c, std::integral_constant<int, 8>{});
        else launch_agg(red_c, std::integral_constant<int, 12>{});
    };
    if (reduce == NGNN_REDUCE_MEAN) by_nc(std::integral_constant<int, NGNN_REDUCE_MEAN>{});
    else if (reduce == NGNN_REDUCE_SUM) by_nc(std::integral_constant<int, NGNN_REDUCE_SUM>{});
    else by_nc(std::integral_constant<int, NGNN_REDUCE_MAX>{});
    return launch_status();
}
}  // namespace ngnn

extern "C" int ngnn_sage_wide_preferred(int64_t K, int64_t Fo, int exact) {
    if (K <= 0 || Fo <= 0) return 0;
    return ngnn::sage_wide_preferred(K, Fo, exact != 0) ? 1 : 0;
}
