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
// Bytes per launch: 4*(N*K + E*K + E + N + 1 + N*F_out) (x, gathered rows,
// col, rowptr, out) + the optional saved aggregate; flops 2*N*K*F_out +
// 2*N_edge_rows*K*F_out.
#include <cstdlib>

#include "ngnn_device.h"

namespace ngnn {

namespace {

constexpr int RT_ROWS = 16;  // rows per wave tile (one MFMA n-tile)
constexpr int RT_KC = 8;     // k-groups of 16 per chunk (128 columns of K)
// waves per workgroup: 2 per SIMD (<= 256 VGPRs: accumulators, the current
// and the prefetched x fragments, two W fragment sets)
// PRE (aggregate precomputed by k_rt_agg, no gather code): fewer live
// registers, so narrow outputs run 4 waves per SIMD to hide the x stream
constexpr int rt_waves(int ntw, bool pre) { return (pre && ntw <= 3) ? 16 : 8; }

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
    Epi epi;
    uint32_t x_bytes, out_bytes, agg_bytes;  // buffer-resource ranges (all < 4 GiB)
    const uint64_t *seed_dev;                 // XORed into the dropout seed (HIP-graph replays)
    const float *const *x_dev;                // non-null: x's address read at run time (graph slot)
    int dbg;  // ablation bits (NGNN_SAGE_ABLATE, profiling only): 1 no MFMA, 2 no stores, 4 no x loads,
             // 8 no epilogue, 16 no weight prologue
};

// -1 (all ones) when a < b, else 0: a lane mask held in a VGPR, built without
// a compare (no SGPR lane-mask pairs to keep live across the tile loop).
// Operands stay far from overflow (|a - b| < 2^31).
__device__ __forceinline__ int lt_mask(int a, int b) { return (a - b) >> 31; }

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

constexpr int kOOB = 0x7ffffff0;  // byte offset past every range: load 0 / drop

// x fragments of one 128-column chunk: lane (rl, q) holds
// x[r][k0 + 16 g + 4 q .. +3]; rows past n_rows read 0 (buffer range).
// Columns past K (which read the next row) are masked by mask_x at the point
// of USE, not here: masking right after the loads would make the compiler
// wait for a prefetch the moment it is issued.
__device__ __forceinline__ void load_x(v4f (&xf)[RT_KC], const RtArgs &a, i32x4 xr, int r, int k0,
                                       int q) {
    const int voff = (r * static_cast<int>(a.ldx) + k0 + 4 * q) * 4;
#pragma unroll
    for (int g = 0; g < RT_KC; ++g) xf[g] = buf_load4(xr, voff + 64 * g, 0, 0);
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
    constexpr int P = NTW >= 8 ? NTW / 4 : 1;
    constexpr int H = NTW / P;
    v4f wb[2][H];
    load_w<NTW, H, LDSW>(wb[0], wsrc, KG, kg0, 0, NT, lane);
#pragma unroll
    for (int s = 0; s < RT_KC * P; ++s) {
        const int g = s / P, p = s % P;
        const int sn = s + 1, gn = sn / P, pn = sn % P;
        if (sn < RT_KC * P) load_w<NTW, H, LDSW>(wb[sn & 1], wsrc, KG, kg0 + gn, pn, NT, lane);
        if (g < nkg) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int h = 0; h < H; ++h)
                    acc[p * H + h] = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[s & 1][h][i], xf[g][i],
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
template <int RED>
__device__ __forceinline__ void gather_chunk(v4f (&ag)[RT_KC], const RtArgs &a, i32x4 xr, int beg,
                                             int deg, int maxdeg, int k0, int nkg, int rl, int q) {
    const float ident = (RED == NGNN_REDUCE_MAX) ? -INFINITY : 0.0f;
#pragma unroll
    for (int g = 0; g < RT_KC; ++g) ag[g] = v4f{ident, ident, ident, ident};
    const int kofs = (k0 + 4 * q) * 4;
    const int ld4 = static_cast<int>(a.ldx) * 4;
#pragma unroll 1
    for (int e0 = 0; e0 < maxdeg; e0 += 16) {
        int cb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = e0 + 4 * q + j;
            cb[j] = a.col[(beg + e) & lt_mask(e, deg)];  // invalid slots read col[0]
        }
        const int ne = min(16, maxdeg - e0);
#pragma unroll 1  // one neighbour pair in flight: keep the register budget
        for (int e4 = 0; 4 * e4 < ne; ++e4) {
            const int srcl = rl + 16 * e4;
#pragma unroll
            for (int j = 0; j < 4; j += 2) {
                const int e = e0 + 4 * e4 + j;
                const int m0 = lt_mask(e, deg), m1 = lt_mask(e + 1, deg);
                const int o0 = m0 ? __shfl(cb[j], srcl) * ld4 + kofs : kOOB;
                const int o1 = m1 ? __shfl(cb[j + 1], srcl) * ld4 + kofs : kOOB;
                // all 8 k-groups unconditionally (conditional writes into the
                // fragment arrays make the compiler copy them whole); groups
                // past K read the next row or 0 and are zeroed at the end
                v4f v0[RT_KC], v1[RT_KC];
#pragma unroll
                for (int g = 0; g < RT_KC; ++g) {
                    v0[g] = buf_load4(xr, o0 + 64 * g, 0, 0);
                    v1[g] = buf_load4(xr, o1 + 64 * g, 0, 0);
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

// epilogue: lane holds output features m*16 + 4q .. +3 of row r.  Stores go
// through a buffer resource (rows past n_rows are dropped by the range);
// `vec` (uniform): F_out a multiple of 16 with 16-B aligned rows -- one
// 16-B store per m-tile, no per-lane predicates.
template <int NTW, bool DROP>
__device__ __forceinline__ void epilogue(const v4f (&acc)[NTW], const RtArgs &a, i32x4 orsrc,
                                         const float *sbias, int r, bool vec, int q) {
    // relu through a wave-uniform select; dropout (hash per element) only in
    // the DROP instantiation
    const uint32_t rk = DROP ? a.epi.drop.row_key(static_cast<uint32_t>(r)) : 0u;
    const int obase = r * static_cast<int>(a.ldo) * 4;
    const bool relu = a.epi.relu;
#pragma unroll
    for (int m = 0; m < NTW; ++m) {
        if (m >= a.NT) continue;  // padded tiles (uniform)
        const int f = m * 16 + 4 * q;
        const v4f b = *reinterpret_cast<const v4f *>(sbias + f);
        // two pair hashes cover the lane's 4 columns (col_base + f is even)
        const uint32_t c0 = static_cast<uint32_t>(a.epi.col_base + f);
        v4f v;
#pragma unroll
        for (int j = 0; j < 4; j += 2) {
            const uint32_t h = DROP ? a.epi.drop.pair_hash(rk, c0 + j) : 0u;
#pragma unroll
            for (int jj = j; jj < j + 2; ++jj) {
                float y = acc[m][jj] + b[jj];
                y = (relu && y < 0.0f) ? 0.0f : y;  // NaN passes, like torch.relu
                if (DROP) y = a.epi.drop.keep_half(h, c0 + jj) ? y * a.epi.drop.scale : 0.0f;
                v[jj] = y;
            }
        }
        if (a.dbg & 2) {
            if (v[0] == 12345.f) buf_store1(v[1], orsrc, obase, 0, 0);  // keep the math alive
        } else if (vec) {
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
template <int NTW, int RED, int WLM, bool PRE>
__global__ __launch_bounds__(rt_waves(NTW, PRE) * 64) void k_sage_rt(RtArgs a) {
    constexpr bool WL_LDS = WLM == 1;
    constexpr int RT_WAVES = rt_waves(NTW, PRE);
    extern __shared__ __attribute__((aligned(16))) v4f lds[];
    const int nfr = NTW * a.KG * 64;  // fragments per weight matrix (NTW tiles, zero padded)
    v4f *swr = lds;
    v4f *swl = lds + nfr;
    float *sbias = reinterpret_cast<float *>(lds + (WL_LDS ? 2 : 1) * nfr);
    const int have_l = a.wl != nullptr;
    {
        // weights -> LDS by LDS-DMA, 1 KiB (one n-tile x k-group fragment)
        // per wave-instruction, all in flight at once; padding tiles zeroed
        const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
        const int nch = (a.dbg & 16) ? 0 : a.NT * a.KG;  // valid 1-KiB chunks per matrix
        for (int c = wv; c < nch; c += RT_WAVES) {
            const int m = c / a.KG, kg = c - m * a.KG;  // [NT][KG] -> LDS [KG][NTW]
            const int d = (kg * NTW + m) * 64;
            bool ok = true;
            const int64_t so = a.ldw ? raw_frag_off(m, kg, ln, a.ldw, a.Fo, a.K, &ok) / 4
                                     : static_cast<int64_t>(c) * 64 + ln;  // in v4f units
            // (raw rows are 16-B aligned: K % 4 == 0 and ldw % 4 == 0)
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(a.wr + so),
                (__attribute__((address_space(3))) void *)(swr + d), 16, 0, 0);
            if (WL_LDS && have_l)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(a.wl + so),
                    (__attribute__((address_space(3))) void *)(swl + d), 16, 0, 0);
        }
        if (a.ldw) {
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
                    swr[d + ln] = z0;
                    if (WL_LDS && have_l) swl[d + ln] = z0;
                }
            }
        }
        const v4f z{0.f, 0.f, 0.f, 0.f};
        const int npad = (NTW - a.NT) * 64;  // padded tiles of every k-group
        for (int i = threadIdx.x; i < a.KG * npad; i += RT_WAVES * 64) {
            const int kg = i / npad, j = i - kg * npad;
            swr[kg * NTW * 64 + a.NT * 64 + j] = z;
            if (WL_LDS) swl[kg * NTW * 64 + a.NT * 64 + j] = z;
        }
        if (WL_LDS && !have_l)
            for (int i = threadIdx.x; i < nfr; i += RT_WAVES * 64) swl[i] = z;
        for (int i = threadIdx.x; i < NTW * 16; i += RT_WAVES * 64)
            sbias[i] = (a.epi.bias && i < a.Fo) ? a.epi.bias[i] : 0.0f;
    }
    __syncthreads();

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q = lane >> 4, rl = lane & 15;
    int n_rows = a.n_rows;
    if (a.n_rows_dev) n_rows = min(n_rows, *a.n_rows_dev);
    int n_tiles = (n_rows + RT_ROWS - 1) / RT_ROWS;
    if (a.tile_end_dev) n_tiles = min(n_tiles, (*a.tile_end_dev + RT_ROWS - 1) / RT_ROWS);
    const int nchunk = (a.KG + RT_KC - 1) / RT_KC;
    const int tstride = gridDim.x * RT_WAVES;

    // tile k of this wave: k = 0 -> w0; later rounds in reverse wave order,
    // so the partial last round lands on the waves that did NOT start with a
    // (heavier) edge tile -- NeighborLoader puts the rows with in-edges
    // first (ablation bit 64 restores the plain order; -0.3..0.4 % step time)
    const int w0 = blockIdx.x + gridDim.x * wave;
    const bool rev = (a.dbg & 64) == 0;
    auto tile_of = [&](int k) { return (k == 0 || !rev) ? w0 + k * tstride : k * tstride + (tstride - 1 - w0); };
    int kt = 0;
    int t = w0;
    if ((a.dbg & 32) && wave >= RT_WAVES / 2) __builtin_amdgcn_s_sleep(100);  // experiment: stagger SIMD partners
    // next tile's chunk-0 x fragments and row bounds, loaded one tile ahead,
    // unconditionally (a tile past the end re-reads tile 0: valid, unused)
    v4f xn[RT_KC];
#pragma unroll
    for (int g = 0; g < RT_KC; ++g) xn[g] = v4f{0.f, 0.f, 0.f, 0.f};
    int nbeg = 0, nend = 0;
    if (a.seed_dev) a.epi.drop.reseed(*a.seed_dev);
    // x: the address given at launch, or (graph replay of a changing batch)
    // the one the slot load stored, ranged by the device row count
    const i32x4 xr = a.x_dev ? make_rsrc(*a.x_dev, static_cast<uint32_t>(
                                             ((n_rows - 1) * a.ldx + a.K) * 4 * (n_rows > 0)))
                             : make_rsrc(a.x, a.x_bytes);
    const i32x4 orsrc = make_rsrc(a.out, a.out_bytes);
    auto prefetch = [&](int tn) {
        const int rn = (tn < n_tiles ? tn : 0) * RT_ROWS + rl;
        if (!(a.dbg & 4)) load_x(xn, a, xr, rn, 0, q);
        if (have_l) {
            const int mr = lt_mask(rn, n_rows);
            const int rr = rn & mr;
            nbeg = a.rowptr[rr];
            nend = a.rowptr[rr + 1];
            nend = nbeg + ((nend - nbeg) & mr);  // rows past the end: degree 0
        }
    };
    const bool vec = a.vec_out && (a.Fo == a.NT * 16);
    prefetch(t);
    for (; t < n_tiles; t = tile_of(++kt)) {
        const int r = t * RT_ROWS + rl;
        const int beg = nbeg, deg = nend - nbeg;
        const int maxdeg = have_l ? rowgroup_max16(deg) : 0;
        v4f acc[NTW];
#pragma unroll
        for (int m = 0; m < NTW; ++m) acc[m] = v4f{0.f, 0.f, 0.f, 0.f};

        // ---- root term: x[r] . W_r^T, chunk by chunk; chunk c+1 (or, in the
        // last chunk, the next tile's chunk 0 and row bounds) loads behind
        // chunk c's MFMAs
        for (int c = 0; c < nchunk; ++c) {
            v4f xc[RT_KC];
            mask_x(xc, xn, a, c * RT_KC * 16, q);
            const int nkg = min(RT_KC, a.KG - c * RT_KC);
            if (c + 1 < nchunk) {
                if (!(a.dbg & 4)) load_x(xn, a, xr, r, (c + 1) * RT_KC * 16, q);
            } else {
                prefetch(tile_of(kt + 1));  // next tile: a whole tile of MFMAs to land
            }
            if (!(a.dbg & 1)) mfma_chunk_rt<NTW, true>(acc, xc, swr, a.KG, c * RT_KC, nkg, a.NT, lane);
        }

        // ---- neighbour term (tiles with in-edges only)
        if (PRE && maxdeg > 0) {
            // aggregate rows written by k_rt_agg (rows with in-edges only;
            // others masked to 0, as the gather's empty-row result)
            const i32x4 ar = make_rsrc(a.agg_out, a.agg_bytes);
            const int mrow = lt_mask(0, deg);
            for (int c = 0; c < nchunk; ++c) {
                const int k0 = c * RT_KC * 16;
                const int nkg = min(RT_KC, a.KG - c * RT_KC);
                const int kq = a.K - k0 - 4 * q;
                const int aoff = (r * static_cast<int>(a.ld_agg) + k0 + 4 * q) * 4;
                v4f ag[RT_KC];
#pragma unroll
                for (int g = 0; g < RT_KC; ++g) ag[g] = buf_load4(ar, aoff + 64 * g, 0, 0);
#pragma unroll
                for (int g = 0; g < RT_KC; ++g) ag[g] = and_mask(ag[g], mrow & lt_mask(16 * g, kq));
                if constexpr (WL_LDS)
                    mfma_chunk_rt<NTW, true>(acc, ag, swl, a.KG, c * RT_KC, nkg, a.NT, lane);
                else
                    mfma_chunk_rt<NTW, false>(acc, ag, a.wl, a.KG, c * RT_KC, nkg, a.NT, lane);
            }
        }
        if (!PRE && maxdeg > 0) {
            const i32x4 ar = make_rsrc(a.agg_out, a.agg_bytes);
            for (int c = 0; c < nchunk; ++c) {
                const int k0 = c * RT_KC * 16;
                const int nkg = min(RT_KC, a.KG - c * RT_KC);
                v4f ag[RT_KC];
                gather_chunk<RED>(ag, a, xr, beg, deg, maxdeg, k0, nkg, rl, q);
                if (a.agg_out) {
                    const int kq = a.K - k0 - 4 * q;
                    const int aoff = (r * static_cast<int>(a.ld_agg) + k0 + 4 * q) * 4;
#pragma unroll
                    for (int g = 0; g < RT_KC; ++g)
                        if (g < nkg) buf_store4(ag[g], ar, 16 * g < kq ? aoff + 64 * g : kOOB, 0, 0);
                }
                if constexpr (WL_LDS)
                    mfma_chunk_rt<NTW, true>(acc, ag, swl, a.KG, c * RT_KC, nkg, a.NT, lane);
                else
                    mfma_chunk_rt<NTW, false>(acc, ag, a.wl, a.KG, c * RT_KC, nkg, a.NT, lane);
            }
        }

        // ---- epilogue (bias, relu, dropout and the stores)
        if (!(a.dbg & 8)) {
            if (a.epi.drop.thresh)
                epilogue<NTW, true>(acc, a, orsrc, sbias, r, vec, q);
            else
                epilogue<NTW, false>(acc, a, orsrc, sbias, r, vec, q);
        }
    }
}

// ---- aggregate pre-pass for the PRE kernels: agg[r] = reduce over the CSR
// row r of x, for rows r < n_rows (and < *n_rows_dev) WITH in-edges only
// (edgeless rows are never written; the layer kernel masks them to 0).  LPR
// lanes per row, 16-B loads, RT_AGG_UNR neighbour rows in flight per group,
// per column in edge order from the identity then / max(deg, 1): the fp32
// sequence of ngnn_seg_agg_fwd, bit-identical.  Rows are interleaved over
// the (resident) grid's groups, so a NeighborLoader block's edge rows (a
// prefix) spread over every CU.
constexpr int RT_AGG_UNR = 8;
template <int RED, int LPR>
__global__ __launch_bounds__(256) void k_rt_agg(const float *__restrict__ x_arg, int64_t ldx, int K,
                                                const int32_t *__restrict__ rowptr,
                                                const int32_t *__restrict__ col, int n_rows,
                                                const int32_t *__restrict__ n_rows_dev,
                                                float *__restrict__ agg, int64_t ld_agg,
                                                const float *const *x_dev, int zero_empty) {
    const float *__restrict__ x = x_dev ? *x_dev : x_arg;
    constexpr int GPW = 256 / LPR;
    const int lane = threadIdx.x % LPR;
    int nr = n_rows;
    if (n_rows_dev) nr = min(nr, *n_rows_dev);
    const int ngroups = gridDim.x * GPW;
    const int gid = blockIdx.x * GPW + threadIdx.x / LPR;
    const float ident = (RED == NGNN_REDUCE_MAX) ? -INFINITY : 0.0f;
    // the group's rows gid + j ngroups, LPR of them per round: lane j loads
    // row j's bounds (one load round for LPR rows, so edgeless rows cost no
    // latency chain), then the group walks the rows that have in-edges
    for (int r0 = gid; r0 < nr; r0 += LPR * ngroups) {
        const int my = r0 + lane * ngroups;
        int mb = 0, me = 0;
        if (my < nr) {
            mb = rowptr[my];
            me = rowptr[my + 1];
        }
        for (int j = 0; j < LPR; ++j) {
        const int beg = __shfl(mb, j, LPR), end = __shfl(me, j, LPR);
        const int row = r0 + j * ngroups;
        if (beg == end) {
            // edgeless row: left unwritten, or zeroed when the caller needs
            // every row (the dense split's agg . W_l^T pass)
            if (zero_empty && row < nr)
                for (int f = 4 * lane; f < K; f += 4 * LPR)
                    *reinterpret_cast<v4f *>(agg + static_cast<int64_t>(row) * ld_agg + f) =
                        v4f{0.f, 0.f, 0.f, 0.f};
            continue;
        }
        for (int f0 = 0; f0 < K; f0 += 4 * LPR) {
            const int f = f0 + 4 * lane;
            const bool act = f < K;
            const int fc = act ? f : 0;
            v4f acc{ident, ident, ident, ident};
            for (int eb = beg; eb < end; eb += LPR) {
                const int n = min(LPR, end - eb);
                const int myc = lane < n ? col[eb + lane] : 0;
                // RT_AGG_UNR rows in flight per batch; a short last batch
                // re-reads its last row (cached) and skips the extra terms
                for (int k = 0; k < n; k += RT_AGG_UNR) {
                    v4f v[RT_AGG_UNR];
#pragma unroll
                    for (int u = 0; u < RT_AGG_UNR; ++u) {
                        const int64_t c = __shfl(myc, min(k + u, n - 1), LPR);
                        v[u] = *reinterpret_cast<const v4f *>(x + c * ldx + fc);
                    }
#pragma unroll
                    for (int u = 0; u < RT_AGG_UNR; ++u)
                        if (k + u < n)
#pragma unroll
                            for (int i = 0; i < 4; ++i) acc[i] = red_op<RED>(acc[i], v[u][i]);
                }
            }
            if (!act) continue;
            if (RED == NGNN_REDUCE_MEAN) {
                const float cnt = static_cast<float>(end - beg);  // deg >= 1 here
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[i] = acc[i] / cnt;
            }
            *reinterpret_cast<v4f *>(agg + static_cast<int64_t>(row) * ld_agg + f) = acc;
        }
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

template <int NTW, int RED, int WLM, bool PRE>
int launch_rt(const RtArgs &a, int n_tiles, size_t lds_bytes, hipStream_t st) {
    auto fn = k_sage_rt<NTW, RED, WLM, PRE>;
    static bool attr_set = false;  // benign race: idempotent
    if (!attr_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(fn),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    constexpr int W = rt_waves(NTW, PRE);
    const int grid = static_cast<int>(
        std::max<int64_t>(1, std::min<int64_t>(num_cus(), ceil_div(n_tiles, W))));
    hipLaunchKernelGGL(fn, dim3(grid), dim3(W * 64), lds_bytes, st, a);
    return launch_status();
}

template <int NTW, bool PRE>
int dispatch_red(const RtArgs &a, int reduce, bool wl_lds, int n_tiles, size_t lds, hipStream_t st) {
    if (PRE)  // the reduction happened in k_rt_agg: one instantiation serves all
        return wl_lds ? launch_rt<NTW, NGNN_REDUCE_SUM, 1, true>(a, n_tiles, lds, st)
                      : launch_rt<NTW, NGNN_REDUCE_SUM, 0, true>(a, n_tiles, lds, st);
    auto by_red = [&](auto red_c) {
        constexpr int RED = decltype(red_c)::value;
        return wl_lds ? launch_rt<NTW, RED, 1, false>(a, n_tiles, lds, st)
                      : launch_rt<NTW, RED, 0, false>(a, n_tiles, lds, st);
    };
    if (reduce == NGNN_REDUCE_MEAN) return by_red(std::integral_constant<int, NGNN_REDUCE_MEAN>{});
    if (reduce == NGNN_REDUCE_SUM) return by_red(std::integral_constant<int, NGNN_REDUCE_SUM>{});
    return by_red(std::integral_constant<int, NGNN_REDUCE_MAX>{});
}

template <int NTW>
int dispatch_pre(const RtArgs &a, int reduce, bool wl_lds, bool pre, int n_tiles, size_t lds,
                 hipStream_t st) {
    return pre ? dispatch_red<NTW, true>(a, reduce, wl_lds, n_tiles, lds, st)
               : dispatch_red<NTW, false>(a, reduce, wl_lds, n_tiles, lds, st);
}

// aggregate of rows [0, min(n_rows, *n_rows_dev)) into agg (edgeless rows
// zeroed), the fp32 sequence of ngnn_seg_agg_fwd
int launch_rt_agg(const float *x, const float *const *x_dev, int64_t ldx, int64_t K,
                  const int32_t *rowptr, const int32_t *col, int64_t n_rows,
                  const int32_t *n_rows_dev, int reduce, float *agg, int64_t ld_agg,
                  hipStream_t st) {
    const int64_t k4 = ceil_div(K, 4);
    const int lpr = k4 <= 8 ? 8 : k4 <= 16 ? 16 : k4 <= 32 ? 32 : 64;
    const unsigned grid = static_cast<unsigned>(
        std::max<int64_t>(1, std::min<int64_t>(8 * num_cus(), ceil_div(n_rows, 256 / lpr))));
    auto go = [&](auto red_c, auto lpr_c) {
        hipLaunchKernelGGL((k_rt_agg<decltype(red_c)::value, decltype(lpr_c)::value>), dim3(grid),
                           dim3(256), 0, st, x, ldx, static_cast<int>(K), rowptr, col,
                           static_cast<int>(n_rows), n_rows_dev, agg, ld_agg, x_dev, 1);
    };
    auto by_lpr = [&](auto red_c) {
        switch (lpr) {
            case 8: go(red_c, std::integral_constant<int, 8>{}); break;
            case 16: go(red_c, std::integral_constant<int, 16>{}); break;
            case 32: go(red_c, std::integral_constant<int, 32>{}); break;
            default: go(red_c, std::integral_constant<int, 64>{}); break;
        }
    };
    if (reduce == NGNN_REDUCE_MEAN) by_lpr(std::integral_constant<int, NGNN_REDUCE_MEAN>{});
    else if (reduce == NGNN_REDUCE_SUM) by_lpr(std::integral_constant<int, NGNN_REDUCE_SUM>{});
    else by_lpr(std::integral_constant<int, NGNN_REDUCE_MAX>{});
    return launch_status();
}

}  // namespace

// Returns 1 and stores the launch status in *rc when the row-tile kernel
// takes this call, 0 when the shape is outside its envelope (the caller then
// runs the 64-row kernel).  Envelope: no input mask, K % 4 == 0 with 16-B
// aligned rows, packed W_r of one column slice fitting in LDS.  Outputs wider
// than one slice (<= 256 columns, fewer when K is large) run as one launch
// per slice; the packed weights are n-tile major, so a slice is a contiguous
// sub-array.
int sage_fwd_rowtile(const float *x, int64_t ldx, int64_t K, int64_t n_rows,
                     const int32_t *n_rows_dev, int64_t tile_end, const int32_t *tile_end_dev,
                     bool prefer_wl_lds, const int32_t *rowptr, const int32_t *col,
                     int reduce, const void *wl_packed, const void *wr_packed, const float *bias,
                     int64_t Fo, float *out, int64_t ldo, int relu, float p_drop, uint64_t seed,
                     const uint64_t *seed_dev, float *agg_out, int64_t ld_agg, hipStream_t st,
                     int *rc, int64_t ldw, void *wl_ws, size_t wl_ws_bytes,
                     const float *const *x_dev) {
    static const bool off = getenv("NGNN_NO_ROWTILE") != nullptr;
    if (off) return 0;
    // (with x_dev the run-time address must be 16-B aligned, as torch's are)
    if (K % 4 != 0 || ldx % 4 != 0 || (!x_dev && !aligned(x, 16))) return 0;
    if (ldw && (ldw % 4 != 0 || !aligned(wr_packed, 16) || (wl_packed && !aligned(wl_packed, 16))))
        return 0;
    if (agg_out && (ld_agg % 4 != 0 || !aligned(agg_out, 16))) return 0;
    // byte offsets are 32-bit (buffer resources): every buffer < 2 GiB
    const int64_t lim = (int64_t(1) << 31) - 4096;
    if (n_rows * ldx * 4 > lim || n_rows * ldo * 4 > lim || (agg_out && n_rows * ld_agg * 4 > lim))
        return 0;
    const int KG = static_cast<int>(ceil_div(K, 16));
    const size_t frag_kb = static_cast<size_t>(KG) * 64 * sizeof(v4f);  // one m-tile, all of K
    const size_t lds_cap = 160 * 1024 - 1024;                          // minus the bias slice
    // widest supported tile count whose W_r fits
    // NGNN_RT_MAXNTW caps the slice width (column tiles per wave) -- tuning experiments
    static const int ntw_cap = getenv("NGNN_RT_MAXNTW") ? atoi(getenv("NGNN_RT_MAXNTW")) : 16;
    int ntw_max = 0;
    for (int c : {16, 8, 4, 3, 2})  // prefer_wl_lds: narrower slices whose W_r AND W_l fit
        if (c <= ntw_cap &&
            static_cast<size_t>(c) * frag_kb * ((prefer_wl_lds && wl_packed) ? 2 : 1) <= lds_cap) {
            ntw_max = c;
            break;
        }
    if (ntw_max == 0) return 0;
    const int64_t slice = 16 * static_cast<int64_t>(ntw_max);
    const Dropout drop = make_dropout(p_drop, seed);
    // PRE (NGNN_RT_PRE=1): the aggregate (saved for the backward anyway) is
    // computed by a separate pass and the layer kernel reads it densely -- no
    // gather registers, 4 waves per SIMD for narrow outputs.  Measured on the
    // products block it loses to the in-kernel gather at both layers (the
    // separate pass re-reads what the gather overlaps: L0 129 + 18 us vs
    // 141 us, L1 60 + 35 us vs 87 us), so the gather stays the default.
    const bool use_pre = getenv("NGNN_RT_PRE") != nullptr;  // read per call (tests toggle it)
    const bool pre = use_pre && agg_out != nullptr && wl_packed != nullptr && rowptr != nullptr;
    if (pre) {
        const int64_t k4 = ceil_div(K, 4);
        const int lpr = k4 <= 8 ? 8 : k4 <= 16 ? 16 : k4 <= 32 ? 32 : 64;
        const unsigned grid = static_cast<unsigned>(
            std::max<int64_t>(1, std::min<int64_t>(8 * num_cus(), ceil_div(n_rows, 256 / lpr))));
        auto go = [&](auto red_c, auto lpr_c) {
            hipLaunchKernelGGL((k_rt_agg<decltype(red_c)::value, decltype(lpr_c)::value>),
                               dim3(grid), dim3(256), 0, st, x, ldx, static_cast<int>(K), rowptr,
                               col, static_cast<int>(n_rows), n_rows_dev, agg_out, ld_agg, x_dev, 0);
        };
        auto by_lpr = [&](auto red_c) {
            switch (lpr) {
                case 8: go(red_c, std::integral_constant<int, 8>{}); break;
                case 16: go(red_c, std::integral_constant<int, 16>{}); break;
                case 32: go(red_c, std::integral_constant<int, 32>{}); break;
                default: go(red_c, std::integral_constant<int, 64>{}); break;
            }
        };
        if (reduce == NGNN_REDUCE_MEAN) by_lpr(std::integral_constant<int, NGNN_REDUCE_MEAN>{});
        else if (reduce == NGNN_REDUCE_SUM) by_lpr(std::integral_constant<int, NGNN_REDUCE_SUM>{});
        else by_lpr(std::integral_constant<int, NGNN_REDUCE_MAX>{});
        const int arc = launch_status();
        if (arc) {
            *rc = arc;
            return 1;
        }
    }
    for (int64_t c0 = 0; c0 < Fo; c0 += slice) {
        const int64_t Fo_c = std::min<int64_t>(slice, Fo - c0);
        const int NT = static_cast<int>(ceil_div(Fo_c, 16));
        const int NTW = NT <= 2 ? 2 : NT <= 3 ? 3 : NT <= 4 ? 4 : NT <= 8 ? 8 : 16;
        const size_t wbytes = static_cast<size_t>(NTW) * frag_kb;
        const size_t bbytes = static_cast<size_t>(NTW) * 16 * sizeof(float);
        // W_l shares the LDS when both fit; otherwise its fragments stream from L2
        const bool wl_lds = wl_packed == nullptr || 2 * wbytes + bbytes <= lds_cap + 1024;
        const size_t lds = (wl_lds ? 2 : 1) * wbytes + bbytes;
        const int64_t toff = (c0 / 16) * KG * 64;
        RtArgs a;
        a.x = x;
        a.ldx = ldx;
        a.K = static_cast<int>(K);
        a.KG = KG;
        a.n_rows = static_cast<int>(n_rows);
        a.n_rows_dev = n_rows_dev;
        a.tile_end_dev = tile_end_dev;
        a.rowptr = rowptr;
        a.col = col;
        // a slice's weights: packed fragments are n-tile major (contiguous
        // sub-array); raw weights are rows [c0, c0 + Fo_c)
        const int64_t woff = ldw ? c0 * ldw / 4 : toff;
        a.wl = wl_packed ? static_cast<const v4f *>(wl_packed) + woff : nullptr;
        a.wr = static_cast<const v4f *>(wr_packed) + woff;
        a.ldw = ldw;
        if (ldw && wl_packed && !wl_lds) {
            // raw W_l that must stream from L2: pack it once (all slices) into
            // the caller's workspace -- fragment-ordered 1-KiB wave loads
            if (c0 == 0) {
                if (!wl_ws || wl_ws_bytes < ngnn_pack_weight_bytes(Fo, K)) {
                    *rc = NGNN_E_WORKSPACE;
                    return 1;
                }
                const int prc = ngnn_pack_weight(static_cast<const float *>(wl_packed), ldw, Fo, K,
                                                 wl_ws, st);
                if (prc) {
                    *rc = prc;
                    return 1;
                }
            }
            a.wl = static_cast<const v4f *>(wl_ws) + toff;
        }
        a.NT = NT;
        a.Fo = static_cast<int>(Fo_c);
        a.out = out + c0;
        a.ldo = ldo;
        a.vec_out = (Fo_c % 4 == 0) && (ldo % 4 == 0) && aligned(out + c0, 16);
        a.agg_out = (pre || c0 == 0) ? agg_out : nullptr;  // PRE: every slice reads it
        a.ld_agg = ld_agg;
        a.epi = Epi{bias ? bias + c0 : nullptr, relu, drop, static_cast<int>(c0)};
        static const int dbg = getenv("NGNN_SAGE_ABLATE") ? atoi(getenv("NGNN_SAGE_ABLATE")) : 0;
        a.dbg = dbg;
        a.seed_dev = seed_dev;
        a.x_dev = x_dev;
        a.x_bytes = static_cast<uint32_t>(((n_rows - 1) * ldx + K) * 4);
        a.out_bytes = static_cast<uint32_t>(((n_rows - 1) * ldo + Fo_c) * 4);
        a.agg_bytes = a.agg_out ? static_cast<uint32_t>(((n_rows - 1) * ld_agg + K) * 4) : 0u;
        const int n_tiles = static_cast<int>(ceil_div(std::min(tile_end, n_rows), RT_ROWS));
        switch (NTW) {
            case 2: *rc = dispatch_pre<2>(a, reduce, wl_lds, pre, n_tiles, lds, st); break;
            case 3: *rc = dispatch_pre<3>(a, reduce, wl_lds, pre, n_tiles, lds, st); break;
            case 4: *rc = dispatch_pre<4>(a, reduce, wl_lds, pre, n_tiles, lds, st); break;
            case 8: *rc = dispatch_pre<8>(a, reduce, wl_lds, pre, n_tiles, lds, st); break;
            default: *rc = dispatch_pre<16>(a, reduce, wl_lds, pre, n_tiles, lds, st); break;
        }
        if (*rc) return 1;
    }
    return 1;
}

}  // namespace ngnn

using namespace ngnn;

// padded row stride of the split path's agg . W_l^T rows
static int64_t split_ldz(int64_t Fo) { return ceil_div(Fo, 16) * 16; }

extern "C" size_t ngnn_sage_fwd_raw_workspace_bytes(int64_t K, int64_t Fo, int64_t n_rows) {
    // a packed W_l (fused path, when it cannot sit in LDS), or the split
    // path's agg . W_l^T rows
    const size_t pack = ngnn_pack_weight_bytes(Fo, K);
    const size_t z = static_cast<size_t>(std::max<int64_t>(n_rows, 0)) * split_ldz(Fo) * sizeof(float);
    return std::max(pack, z);
}

extern "C" int ngnn_sage_fwd_raw(const float *x, const float *const *x_dev, int64_t ldx,
                                 int64_t K, int64_t n_rows, const int32_t *n_rows_dev,
                                 int64_t n_edge_rows, const int32_t *n_edge_rows_dev,
                                 const int32_t *rowptr,
                                 const int32_t *col, int reduce, const float *wl, const float *wr,
                                 int64_t ldw, const float *bias, int64_t Fo, float *out,
                                 int64_t ldo, int relu, float p_drop, uint64_t seed,
                                 const uint64_t *seed_dev, float *agg_out, int64_t ld_agg, void *ws,
                                 size_t ws_bytes, void *stream) {
    NGNN_RETURN_IF(reduce < NGNN_REDUCE_SUM || reduce > NGNN_REDUCE_MAX, NGNN_E_ARG);
    NGNN_RETURN_IF(K <= 0 || Fo <= 0 || n_rows < 0 || !wr, NGNN_E_ARG);
    NGNN_RETURN_IF(wl && !rowptr, NGNN_E_ARG);
    NGNN_RETURN_IF(ldx < K || ldo < Fo || ldw < K, NGNN_E_SHAPE);
    NGNN_RETURN_IF(agg_out && ld_agg < K, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(K) || !fits_i32(n_rows) || !fits_i32(Fo), NGNN_E_RANGE);
    NGNN_RETURN_IF(p_drop < 0.0f || !(p_drop <= 1.0f), NGNN_E_ARG);
    if (n_rows == 0) return NGNN_OK;
    NGNN_RETURN_IF((!x && !x_dev) || !out, NGNN_E_ARG);
    hipStream_t st = as_stream(stream);
    int rc = NGNN_OK;
    // rows >= the edge-row bound have no in-edges.  No neighbour term: the
    // dense kernel takes every row.  Wide outputs (MFMA-bound) with a known
    // bound: three launches -- the aggregate of the edge rows (saved for the
    // backward anyway), z = agg . W_l^T on those rows (dense kernel, no
    // epilogue), then the dense kernel over every row with z added to the
    // edge rows.  Otherwise the fused gather kernel takes the layer.
    int64_t split = std::max<int64_t>(0, std::min(n_edge_rows, n_rows));
    const int32_t *split_dev = n_edge_rows_dev;
    // opt-in (NGNN_SPLIT=1): measured on products [15,10] L0 the three
    // launches (agg 16 k rows + z + dense 153 k rows) tie the fused kernel
    // (159 vs 155 us): the one-wave-per-SIMD dense kernel reaches ~60 % of the
    // fp32 MFMA rate, not enough to pay for the separate aggregate pass
    const char *split_env = getenv("NGNN_SPLIT");  // read per call (tests toggle it)
    const int split_mode = split_env ? atoi(split_env) : 0;
    if (!wl) {
        if (sage_fwd_dense(x, x_dev, ldx, K, 0, nullptr, n_rows, n_rows_dev, wr, ldw, bias, Fo, out,
                           ldo, relu, p_drop, seed, seed_dev, st, &rc))
            return rc;
    } else if (split_mode == 1 && Fo > 128 && (split < n_rows || split_dev) && agg_out &&
               ws_bytes >= ngnn_sage_fwd_raw_workspace_bytes(K, Fo, n_rows) && aligned(ws, 16) &&
               ld_agg % 4 == 0 && aligned(agg_out, 16)) {
        const int64_t zrows = split_dev ? n_rows : split;  // host bound of the z rows
        float *z = static_cast<float *>(ws);
        const int64_t ldz = split_ldz(Fo);
        const int32_t *zdev = split_dev;
        // the dense kernel's envelope check launches nothing when it refuses,
        // so probe the cheap pass shapes first: z pass and main pass share it
        int rz = NGNN_OK;
        if (zrows > 0 || split_dev) {
            rc = launch_rt_agg(x, x_dev, ldx, K, rowptr, col, zrows, zdev, reduce, agg_out, ld_agg, st);
            if (rc) return rc;
            if (!sage_fwd_dense(agg_out, nullptr, ld_agg, K, 0, nullptr, zrows, zdev, wl, ldw,
                                nullptr, Fo, z, ldz, 0, 0.0f, 0, nullptr, st, &rz))
                goto fused;  // (the agg pass already ran: harmless, the fused kernel rewrites it)
            if (rz) return rz;
        }
        if (sage_fwd_dense(x, x_dev, ldx, K, 0, nullptr, n_rows, n_rows_dev, wr, ldw, bias, Fo, out,
                           ldo, relu, p_drop, seed, seed_dev, st, &rc, z, ldz, zrows, zdev))
            return rc;
    }
fused:
    if (wl && split_mode == 2 && (split < n_rows || split_dev)) {
        // split mode 2: the fused gather kernel on the tiles below the split
        // (output slices narrow enough for W_r and W_l to share the LDS),
        // the dense kernel from the next 16-row boundary up
        const int64_t s16 = std::min(n_rows, ceil_div(split, 16) * 16);
        int rd = NGNN_OK;
        if (sage_fwd_dense(x, x_dev, ldx, K, split_dev ? 0 : s16, split_dev, n_rows, n_rows_dev, wr,
                           ldw, bias, Fo, out, ldo, relu, p_drop, seed, seed_dev, st, &rd, nullptr, 0,
                           0, nullptr, /*round_begin16=*/true)) {
            if (rd) return rd;
            if (!sage_fwd_rowtile(x, ldx, K, n_rows, n_rows_dev, split_dev ? n_rows : s16, split_dev,
                                  true, rowptr, col, reduce, wl, wr, bias, Fo, out, ldo, relu, p_drop,
                                  seed, seed_dev, agg_out, ld_agg, st, &rc, ldw, ws, ws_bytes, x_dev))
                return NGNN_E_SHAPE;
            return rc;
        }
    }
    if (!sage_fwd_rowtile(x, ldx, K, n_rows, n_rows_dev, n_rows, nullptr, false, rowptr, col, reduce,
                          wl, wr,
                          bias, Fo, out, ldo, relu, p_drop, seed, seed_dev, agg_out, ld_agg, st, &rc,
                          ldw, ws, ws_bytes, x_dev))
        return NGNN_E_SHAPE;  // outside the row-tile envelope: pack + ngnn_sage_fwd
    return rc;
}
