// Dense row-tile layer kernel for the rows of a block that have NO in-edges.
//
// A NeighborLoader block numbers the rows that receive edges first (the seeds
// and every hop's frontier but the last): on a products [15,10] block only
// ~16 k of ~153 k rows have in-edges.  Every other row of SAGEConv.forward
// (sage.py:33-39) reduces to
//     out[r] = act(b + x[r] . W_r^T)          (agg(r) = 0, so no W_l term)
// which is a plain GEMM + epilogue with no gather.  ngnn_sage_fwd_raw splits
// the layer there: the fused gather kernel (ngnn_sage_rt.hip) takes the rows
// below the split, this kernel the rows above it.
//
// Design (gfx950, fp32 MFMA-bound at K = 100 -> 256):
//   * one 256-thread workgroup per CU -- ONE wave per SIMD -- persistent;
//     W_r (raw PyG [F_out, K] rows) DMA'd once into LDS in MFMA fragment order
//     [k-group][n-tile][lane] (1 KiB per fragment), bias too;
//   * a wave owns 32-row tiles (two 16-row MFMA sub-tiles sharing every W
//     fragment read); B = x (straight from HBM into registers, the next
//     tile's loads issued before this tile's MFMAs),
//     A = W from LDS, v_mfma_f32_16x16x4_f32, so each lane ends with 4
//     consecutive output features of one row -> 16-B stores;
//   * software pipeline: the epilogue of tile t-1 (bias, ReLU, hash
//     dropout, stores) is spread over the MFMA steps of tile t in one basic
//     block (K is a template constant: no branches in the tile body), so its VALU work and stores issue in the
//     matrix pipe's shadow instead of after it (the fused kernel runs two
//     waves per SIMD whose epilogues do not overlap their partner's MFMAs:
//     tools/ablate.sh measured +26 % over its MFMA-only time on L0).
//
// Bytes per launch: 4 (R K + R F_out) for R rows; flops 2 R K F_out.
#include <algorithm>

#include "ngnn_device.h"

namespace ngnn {

namespace {

constexpr int DN_WAVES = 4;  // one wave per SIMD
// 16-row MFMA sub-tiles per tile (each W fragment feeds 4 RS MFMAs): two for
// the wide (MFMA-bound) outputs, one for narrow outputs, where the x stream
// dominates and lower register use buys more waves per SIMD
constexpr int dn_rs(int ntw) { return ntw >= 32 ? 2 : 1; }

struct DenseArgs {
    const float *x;
    const float *const *x_dev;  // non-null: x's address read at run time (graph slot)
    int64_t ldx;
    int K, KG;
    int row_begin;
    const int32_t *row_begin_dev;  // non-null: first row read at run time
    int round16;                   // first row rounded up to a multiple of 16
    int n_rows;
    const int32_t *n_rows_dev;
    const float *w;  // raw PyG weights [F_out, K], row stride ldw
    int64_t ldw;
    int Fo, NT;
    const float *bias;
    Epi epi;
    const uint64_t *seed_dev;
    float *out;
    int64_t ldo;
    int vec_out;
    uint32_t x_bytes, out_bytes;
    // optional addend (pre-activation partial sums, e.g. agg . W_l^T of the
    // rows that have in-edges): rows < its range add z[r]; rows past it read 0
    const float *z;
    int64_t ldz;  // multiple of 4, >= NTW * 16 (padded n-tiles read it)
    int z_rows;
    const int32_t *z_rows_dev;
};

__device__ __forceinline__ int dn_lt_mask(int a, int b) { return (a - b) >> 31; }

__device__ __forceinline__ v4f dn_and_mask(v4f v, int m) {
    v4f o;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = __int_as_float(__float_as_int(v[i]) & m);
    return o;
}

// epilogue of one n-tile of a finished tile: lane (rl, q) holds output
// features m*16 + 4q .. +3 of row `row` (row >= n_rows: the store offset lies
// past the buffer range and is dropped)
template <bool DROP>
__device__ __forceinline__ void dn_epi_tile(const v4f &acc, const DenseArgs &a, i32x4 orsrc,
                                            const float *sbias, int m, int q, int obase,
                                            uint32_t rk, bool vec) {
    const int f = m * 16 + 4 * q;
    const v4f b = *reinterpret_cast<const v4f *>(sbias + f);
    const uint32_t c0 = static_cast<uint32_t>(a.epi.col_base + f);  // even: pair hashes
    const uint32_t h0 = DROP ? a.epi.drop.pair_hash(rk, c0) : 0u;
    const uint32_t h1 = DROP ? a.epi.drop.pair_hash(rk, c0 + 2) : 0u;
    v4f v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        float y = acc[j] + b[j];
        y = (a.epi.relu && y < 0.0f) ? 0.0f : y;  // NaN passes, like torch.relu
        if (DROP)
            y = ((j & 1) ? a.epi.drop.keep_par<1>(j < 2 ? h0 : h1) : a.epi.drop.keep_par<0>(j < 2 ? h0 : h1))
                    ? y * a.epi.drop.scale
                    : 0.0f;
        v[j] = y;
    }
    if (vec) {  // (F_out % 16 == 0: padded n-tiles start at f >= F_out and are dropped)
        buf_store4(v, orsrc, f < a.Fo ? obase + 4 * f : kBufOOB, 0, 0);
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            buf_store1(v[j], orsrc, f + j < a.Fo ? obase + 4 * (f + j) : kBufOOB, 0, 0);
    }
}

// NTW: n-tiles (16 output columns each, >= NT, padded tiles hold zero W);
// KG: k-groups of 16 columns of K, exact, so the whole tile body is one basic
// block: the MFMAs run in steps of MB n-tiles (W fragments of the next step
// read from LDS while the current step's 4*RS*MB MFMAs issue; RS*MB
// independent accumulators between dependent MFMAs) and the pending tile's
// epilogue is spread over the first steps, interleaved MFMA by MFMA
// (sched_group_barrier).
template <int NTW, int KG, bool DROP, bool ADD>
__global__ __launch_bounds__(DN_WAVES * 64) void k_dense(DenseArgs a) {
    constexpr int RS = dn_rs(NTW);
    constexpr int DN_TROWS = 16 * RS;
    constexpr int MB = NTW >= 4 ? 4 : NTW;  // n-tiles per MFMA step
    constexpr int NB = NTW / MB;            // steps per k-group
    constexpr int NS = KG * NB;             // steps per tile
    extern __shared__ __attribute__((aligned(16))) v4f lds[];
    v4f *sw = lds;
    float *sbias = reinterpret_cast<float *>(lds + KG * NTW * 64);
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    {
        // W -> LDS by LDS-DMA, one 1-KiB fragment (n-tile m, k-group kg) per
        // wave-instruction: lane l brings W[m*16 + (l & 15)][kg*16 + 4 (l >> 4) .. +3]
        const int nch = a.NT * KG;
        for (int c = wv; c < nch; c += DN_WAVES) {
            const int m = c / KG, kg = c - m * KG;
            const int n = m * 16 + (ln & 15), k = kg * 16 + 4 * (ln >> 4);
            const int64_t so = (n < a.Fo && k < a.K) ? static_cast<int64_t>(n) * a.ldw + k : 0;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(a.w + so),
                (__attribute__((address_space(3))) void *)(sw + (kg * NTW + m) * 64), 16, 0, 0);
        }
        __builtin_amdgcn_s_waitcnt(0);  // this wave's LDS-DMAs have landed
        const v4f z{0.f, 0.f, 0.f, 0.f};
        for (int c = wv; c < nch; c += DN_WAVES) {  // lanes outside F_out x K -> 0
            const int m = c / KG, kg = c - m * KG;
            const int n = m * 16 + (ln & 15), k = kg * 16 + 4 * (ln >> 4);
            if (!(n < a.Fo && k < a.K)) sw[(kg * NTW + m) * 64 + ln] = z;
        }
        const int npad = (NTW - a.NT) * 64;  // padded n-tiles of every k-group
        for (int i = threadIdx.x; i < KG * npad; i += DN_WAVES * 64) {
            const int kg = i / npad, j = i - kg * npad;
            sw[kg * NTW * 64 + a.NT * 64 + j] = z;
        }
        for (int i = threadIdx.x; i < NTW * 16; i += DN_WAVES * 64)
            sbias[i] = (a.bias && i < a.Fo) ? a.bias[i] : 0.0f;
    }
    __syncthreads();

    const int lane = ln, q = lane >> 4, rl = lane & 15;
    int rb = a.row_begin;
    if (a.row_begin_dev) rb = *a.row_begin_dev;
    if (a.round16) rb = (rb + 15) & ~15;
    int nr = a.n_rows;
    if (a.n_rows_dev) nr = min(nr, *a.n_rows_dev);
    rb = __builtin_amdgcn_readfirstlane(rb);
    nr = __builtin_amdgcn_readfirstlane(nr);
    const int n_tiles = nr > rb ? (nr - rb + DN_TROWS - 1) / DN_TROWS : 0;
    const int tstride = gridDim.x * DN_WAVES;
    if (a.seed_dev) a.epi.drop.reseed(*a.seed_dev);
    const i32x4 xr = a.x_dev ? make_rsrc_u(*a.x_dev, static_cast<uint32_t>(
                                               ((nr - 1) * a.ldx + a.K) * 4 * (nr > 0)))
                             : make_rsrc_u(a.x, a.x_bytes);
    const i32x4 orsrc = make_rsrc_u(a.out, a.out_bytes);
    i32x4 zr{0, 0, 0, 0};
    if constexpr (ADD) {  // z rows < the addend's row count (device or host), the rest read 0
        int zrows = a.z_rows;
        if (a.z_rows_dev) zrows = min(zrows, *a.z_rows_dev);
        zrows = __builtin_amdgcn_readfirstlane(zrows);
        zr = make_rsrc_u(a.z, static_cast<uint32_t>(zrows > 0 ? zrows * a.ldz * 4 : 0));
    }
    const bool vec = a.vec_out && (a.Fo == a.NT * 16);
    const int kq = a.K - 4 * q;  // group g's 4 columns of this lane are valid iff 16 g < kq

    // x fragments of a tile: lane (rl, q) holds x[r][16 g + 4 q .. +3];
    // rows past nr read 0 (buffer range); a tile past the end re-reads the
    // first tile (valid addresses, never used)
    auto load_x = [&](v4f (&xf)[KG], int tt, int u) {
        const int r = rb + (tt < n_tiles ? tt : 0) * DN_TROWS + 16 * u + rl;
        const int voff = (r * static_cast<int>(a.ldx) + 4 * q) * 4;
#pragma unroll
        for (int g = 0; g < KG; ++g) xf[g] = buf_load4(xr, voff + 64 * g, 0, 0);
    };
    // addend fragments of a tile in the accumulator layout: lane (rl, q)
    // holds z[r][16 m + 4 q .. +3]
    auto load_z = [&](v4f (&zf)[NTW], int tt, int u) {
        const int r = rb + (tt < n_tiles ? tt : 0) * DN_TROWS + 16 * u + rl;
        const int voff = (r * static_cast<int>(a.ldz) + 4 * q) * 4;
#pragma unroll
        for (int m = 0; m < NTW; ++m) zf[m] = buf_load4(zr, voff + 64 * m, 0, 0);
    };
    auto load_w = [&](v4f (&w)[MB], int s) {
        const int g = s / NB, b = s % NB;
#pragma unroll
        for (int h = 0; h < MB; ++h) w[h] = sw[(g * NTW + b * MB + h) * 64 + lane];
    };

    int t = blockIdx.x + gridDim.x * wv;  // consecutive tiles spread over the CUs
    v4f xn[RS][KG];
    v4f zn[RS][ADD ? NTW : 1];
#pragma unroll
    for (int u = 0; u < RS; ++u) {
        load_x(xn[u], t, u);
        if constexpr (ADD) load_z(zn[u], t, u);
    }

    // the pending (previous) tile: accumulators + its rows; the first
    // iteration's "pending" tile is a dummy whose stores fall past the range
    v4f pend[RS][NTW];
#pragma unroll
    for (int u = 0; u < RS; ++u)
#pragma unroll
        for (int m = 0; m < NTW; ++m) pend[u][m] = v4f{0.f, 0.f, 0.f, 0.f};
    int prow = nr;  // first row of the pending tile (lane's rows: prow + 16 u + rl)
    // pending epilogue: EPS (sub-tile, n-tile) pieces after each of the first steps
    constexpr int NPIECE = RS * NTW;
    constexpr int EPS = (NPIECE + NS - 1) / NS;

    for (; t < n_tiles; t += tstride) {
        const int r0 = rb + t * DN_TROWS;
        v4f xc[RS][KG];
#pragma unroll
        for (int u = 0; u < RS; ++u)
#pragma unroll
            for (int g = 0; g < KG; ++g) xc[u][g] = dn_and_mask(xn[u][g], dn_lt_mask(16 * g, kq));
        v4f acc[RS][NTW];
#pragma unroll
        for (int u = 0; u < RS; ++u)
#pragma unroll
            for (int m = 0; m < NTW; ++m) {
                if constexpr (ADD) acc[u][m] = zn[u][m];
                else acc[u][m] = v4f{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
        for (int u = 0; u < RS; ++u) {
            load_x(xn[u], t + tstride, u);
            if constexpr (ADD) load_z(zn[u], t + tstride, u);
        }

        uint32_t rk[RS];
        int obase[RS];
#pragma unroll
        for (int u = 0; u < RS; ++u) {
            const int pr = prow + 16 * u + rl;
            rk[u] = DROP ? a.epi.drop.row_key(static_cast<uint32_t>(pr)) : 0u;
            obase[u] = pr < nr ? pr * static_cast<int>(a.ldo) * 4 : kBufOOB;
        }
        v4f wb[2][MB];
        load_w(wb[0], 0);
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if (s + 1 < NS) load_w(wb[(s + 1) & 1], s + 1);
            const int g = s / NB, b = s % NB;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int u = 0; u < RS; ++u)
#pragma unroll
                    for (int h = 0; h < MB; ++h)
                        acc[u][b * MB + h] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                            wb[s & 1][h][i], xc[u][g][i], acc[u][b * MB + h], 0, 0, 0);
#pragma unroll
            for (int e = 0; e < EPS; ++e) {
                const int piece = s * EPS + e;  // (padded n-tiles: every store dropped)
                if (piece < NPIECE) {
                    const int u = piece / NTW, m = piece % NTW;
                    dn_epi_tile<DROP>(pend[u][m], a, orsrc, sbias, m, q, obase[u], rk[u], vec);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < RS; ++u)
#pragma unroll
            for (int m = 0; m < NTW; ++m) pend[u][m] = acc[u][m];
        prow = r0;
    }
    {  // drain: the last tile's epilogue
#pragma unroll
        for (int u = 0; u < RS; ++u) {
            const int pr = prow + 16 * u + rl;
            const uint32_t rk = DROP ? a.epi.drop.row_key(static_cast<uint32_t>(pr)) : 0u;
            const int obase = pr < nr ? pr * static_cast<int>(a.ldo) * 4 : kBufOOB;
#pragma unroll
            for (int m = 0; m < NTW; ++m)
                if (m < a.NT) dn_epi_tile<DROP>(pend[u][m], a, orsrc, sbias, m, q, obase, rk, vec);
        }
    }
}

int g_dn_cus[64];

int dn_num_cus() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) return 256;
    if (!g_dn_cus[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        g_dn_cus[dev] = n;
    }
    return g_dn_cus[dev];
}

template <int NTW, int KG, bool DROP, bool ADD>
int dn_launch(const DenseArgs &a, int max_tiles, size_t lds, hipStream_t st) {
    auto fn = k_dense<NTW, KG, DROP, ADD>;
    static int per_cu = 0;  // benign race: idempotent
    if (!per_cu) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(fn),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        int occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, DN_WAVES * 64, lds) != hipSuccess ||
            occ <= 0)
            occ = 1;
        per_cu = occ;
    }
    // LDS can cap residency below the register limit for this call's size
    const int by_lds = static_cast<int>(std::max<size_t>(1, (160 * 1024) / std::max<size_t>(lds, 1)));
    const int64_t cap = static_cast<int64_t>(dn_num_cus()) * std::min(per_cu, by_lds);
    const int grid = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(cap, ceil_div(max_tiles, DN_WAVES))));
    hipLaunchKernelGGL(fn, dim3(grid), dim3(DN_WAVES * 64), lds, st, a);
    return launch_status();
}

template <int NTW, int KG>
int dn_drop(const DenseArgs &a, int max_tiles, size_t lds, hipStream_t st) {
    return a.epi.drop.thresh ? dn_launch<NTW, KG, true, false>(a, max_tiles, lds, st)
                             : dn_launch<NTW, KG, false, false>(a, max_tiles, lds, st);
}

template <int NTW, int KG>
int dn_drop_add(const DenseArgs &a, int max_tiles, size_t lds, hipStream_t st) {
    if (!a.z) return dn_drop<NTW, KG>(a, max_tiles, lds, st);
    return a.epi.drop.thresh ? dn_launch<NTW, KG, true, true>(a, max_tiles, lds, st)
                             : dn_launch<NTW, KG, false, true>(a, max_tiles, lds, st);
}

// instantiated (n-tiles, k-groups): the products / arxiv layer shapes --
// K in (96, 128] -> F_out in (240, 256], and K in (240, 256] -> F_out <= 64 or
// in (112, 128]; other shapes take the fused kernel
constexpr bool dn_shape_ok(int ntw, int kg) {
    return (ntw == 16 && (kg == 7 || kg == 8)) || (kg == 16 && (ntw == 3 || ntw == 4 || ntw == 8));
}

}  // namespace

// Returns 1 (launch status in *rc) when the dense kernel takes rows
// [row_begin, n_rows) of this layer, 0 when the shape is outside its
// envelope: K % 4 == 0 with 16-B aligned rows, 48 < K <= 256, F_out <= 256,
// W_r fitting in LDS.
int sage_fwd_dense(const float *x, const float *const *x_dev, int64_t ldx, int64_t K,
                   int64_t row_begin, const int32_t *row_begin_dev, int64_t n_rows,
                   const int32_t *n_rows_dev, const float *wr, int64_t ldw, const float *bias,
                   int64_t Fo, float *out, int64_t ldo, int relu, float p_drop, uint64_t seed,
                   const uint64_t *seed_dev, hipStream_t st, int *rc, const float *z,
                   int64_t ldz, int64_t z_rows, const int32_t *z_rows_dev, bool round_begin16) {
    if (getenv("NGNN_NO_DENSE")) return 0;
    if (K % 4 != 0 || ldx % 4 != 0 || ldw % 4 != 0 || K <= 48 || K > 256 || Fo > 256) return 0;
    if ((!x_dev && !aligned(x, 16)) || !aligned(wr, 16)) return 0;
    const int64_t lim = (int64_t(1) << 31) - 4096;
    if (n_rows * ldx * 4 > lim || (n_rows + 1) * ldo * 4 > lim) return 0;
    const int KG = static_cast<int>(ceil_div(K, 16));
    const int NT = static_cast<int>(ceil_div(Fo, 16));
    const int NTW = NT <= 3 ? 3 : NT <= 4 ? 4 : NT <= 8 ? 8 : 16;
    if (!dn_shape_ok(NTW, KG)) return 0;
    if (z && (NTW != 16 || ldz % 4 != 0 || ldz < NTW * 16 || !aligned(z, 16) ||
              (z_rows + 1) * ldz * 4 > lim))
        return 0;  // (the addend is only instantiated for the wide layers)
    const size_t lds = static_cast<size_t>(KG) * NTW * 64 * sizeof(v4f) + NTW * 16 * sizeof(float);
    if (lds > 160 * 1024) return 0;
    DenseArgs a;
    a.x = x;
    a.x_dev = x_dev;
    a.ldx = ldx;
    a.K = static_cast<int>(K);
    a.KG = KG;
    a.row_begin = static_cast<int>(row_begin);
    a.row_begin_dev = row_begin_dev;
    a.round16 = round_begin16;
    a.n_rows = static_cast<int>(n_rows);
    a.n_rows_dev = n_rows_dev;
    a.w = wr;
    a.ldw = ldw;
    a.Fo = static_cast<int>(Fo);
    a.NT = NT;
    a.bias = bias;
    a.epi = Epi{bias, relu, make_dropout(p_drop, seed), 0};
    a.seed_dev = seed_dev;
    a.out = out;
    a.ldo = ldo;
    a.vec_out = (Fo % 4 == 0) && (ldo % 4 == 0) && aligned(out, 16);
    a.x_bytes = static_cast<uint32_t>(n_rows > 0 ? ((n_rows - 1) * ldx + K) * 4 : 0);
    a.out_bytes = static_cast<uint32_t>(n_rows > 0 ? ((n_rows - 1) * ldo + Fo) * 4 : 0);
    a.z = z;
    a.ldz = ldz;
    a.z_rows = static_cast<int>(z_rows);
    a.z_rows_dev = z_rows_dev;
    const int max_tiles = static_cast<int>(ceil_div(std::max<int64_t>(n_rows - (row_begin_dev ? 0 : row_begin), 0),
                                                    16 * dn_rs(NTW)));
    if (NTW == 16)
        *rc = KG == 7 ? dn_drop_add<16, 7>(a, max_tiles, lds, st)
                      : dn_drop_add<16, 8>(a, max_tiles, lds, st);
    else if (NTW == 3)
        *rc = dn_drop<3, 16>(a, max_tiles, lds, st);
    else if (NTW == 4)
        *rc = dn_drop<4, 16>(a, max_tiles, lds, st);
    else
        *rc = dn_drop<8, 16>(a, max_tiles, lds, st);
    return 1;
}

}  // namespace ngnn
