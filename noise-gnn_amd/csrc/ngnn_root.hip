// k_root: the row-tile SAGEConv forward of the tiles whose rows have no
// in-edges (NeighborLoader numbers the rows that receive edges first, so on a
// products [15,10] block ~90 % of layer 0's 16-row tiles and every tile of the
// narrow output layer), out = act(b + x W_r^T) (narrow: also z = x W_l^T).
//
// Why a second kernel: k_sage_rt runs two 8-wave-per-CU waves per SIMD that
// take turns between a 300-MFMA root term and a VALU/store epilogue; both
// waves of a SIMD reach their MFMAs together, the W-part LDS reads are
// double-buffered one output tile ahead only (~100 cycles to cover an LDS
// round trip at 8 waves), and the MFMA pipe stayed ~50 % busy (PMC:
// SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES, SQ_WAIT_INST_ANY at half the wave
// cycles).  Here ONE wave per SIMD (256-thread workgroups, up to 512 VGPR +
// AGPR per lane) owns the matrix pipe; its W reads run TWO output-tile steps
// ahead through a 3-slot ring, and the next tile's x rows are in flight for a
// whole tile.  Every loop bound (32-column chunks CC, fp32 tail steps T4,
// output tiles NTW) and the epilogue form are compile-time, so a tile is one
// straight-line block.  Same arithmetic, in the same order, as k_sage_rt's
// root term (the split-bf16 products, the tail first, the bias as the
// accumulators' start): the two kernels produce identical bits.
#include "ngnn_sage_rt_kern.h"

#ifndef NGNN_ROOT_NOLOAD
#define NGNN_ROOT_NOLOAD 0
#endif
#ifndef NGNN_ROOT_TRACE
#define NGNN_ROOT_TRACE 0  // (diagnostic builds only) per-segment s_memtime sums
#endif

namespace ngnn {
#if NGNN_ROOT_TRACE
__device__ unsigned long long g_root_trace[8];
#endif
namespace {

constexpr int RR_WAVES = 4;  // one wave per SIMD

__device__ __forceinline__ unsigned long long rr_clock() {
#if NGNN_ROOT_TRACE
    return __builtin_amdgcn_s_memtime();
#else
    return 0;
#endif
}

template <int NTW, int CC, int T4, int FORM, bool XB, bool W1, bool VEC>
__global__ __launch_bounds__(RR_WAVES * 64) __attribute__((amdgpu_waves_per_eu(1, 1))) void k_root(RtArgs a) {
    constexpr int NP = W1 ? 1 : 3;  // weight parts in the image
    constexpr int FB = FORM > 4 ? FORM - 4 : FORM;
    constexpr int DM = FB == 1 ? 2 : 0;
    constexpr bool RELU = FB == 1 || FB == 2, OB = FORM > 4, NAR = FB == 4;
    constexpr uint32_t EB = XB ? 2u : 4u;  // bytes per x element
    constexpr int NG = (CC + 3) / 4;       // 128-column x groups
    constexpr int NXF = NG * RT_KC;        // x fragments per lane (X3 layout)
    constexpr int NSTEP = CC * NTW;        // (32-column chunk, output tile) steps
    constexpr int T4N = T4 > 0 ? T4 : 1;
    static_assert(!NAR || (NTW % 2 == 0 && !OB), "narrow: out / z halves");
    extern __shared__ __attribute__((aligned(16))) v4f lds[];
    __shared__ int s_next;  // the workgroup's tile-claim counter
    [[maybe_unused]] const unsigned long long k0 = rr_clock();
#ifdef NGNN_DBG_EMPTY
    if (a.K != 1234567) return;  // (diagnostic: launch cost alone)
#endif
    if (threadIdx.x == 0) s_next = RR_WAVES;
    const int pst = CC * NTW * 64;  // bf16x8 per weight part
    bf16x8 *sw3 = reinterpret_cast<bf16x8 *>(lds);
    float *swt = reinterpret_cast<float *>(lds + NP * pst);
    float *sbias = swt + T4 * NTW * 64;
    if (a.img) dma_image(lds, a.img, NP * pst, T4 * NTW * 64, RR_WAVES);
    else build_x3_image<NTW, W1>(a, sw3, swt, pst, RR_WAVES * 64);
    for (int i = threadIdx.x; i < NTW * 16; i += RR_WAVES * 64)
        sbias[i] = (a.epi.bias && i < a.Fo) ? a.epi.bias[i] : 0.0f;
    if (a.img) __builtin_amdgcn_s_waitcnt(0);  // (the image's LDS-DMAs landed)
    __syncthreads();

    [[maybe_unused]] const unsigned long long k1 = rr_clock();
#ifdef NGNN_DBG_PROLOGUE_ONLY
    if (k1 != 1234567ull) return;  // (diagnostic: the image build alone)
#endif
    // (run-time values read from device words, made provably wave-uniform:
    // a value the compiler takes for divergent puts the buffer resources in
    // VGPRs and wraps every load and store in a waterfall loop behind an
    // s_waitcnt vmcnt(0) -- a drain of the previous tile's stores per load)
    int n_rows = a.n_rows;
    if (a.n_rows_dev) n_rows = min(n_rows, *a.n_rows_dev);
    n_rows = __builtin_amdgcn_readfirstlane(n_rows);
    const int n_tiles = (n_rows + RT_ROWS - 1) / RT_ROWS;
    // (no neighbour term in the layer -- narrow mode: every tile is a root tile)
    int ne = a.wl ? a.n_edge : 0;
    if (a.wl && a.n_edge_dev) ne = min(ne, *a.n_edge_dev);
    const int t2 = __builtin_amdgcn_readfirstlane(min(n_tiles, (max(ne, 0) + RT_ROWS - 1) / RT_ROWS));
    const int wv = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    // tiles t2 + blockIdx.x + j gridDim.x of this workgroup, claimed one at a
    // time by its waves (the first RR_WAVES fixed)
    auto claim = [&]() __attribute__((always_inline)) -> int {
        int j = 0;
        if ((threadIdx.x & 63) == 0) j = atomicAdd(&s_next, 1);
        return t2 + static_cast<int>(blockIdx.x) +
               __builtin_amdgcn_readfirstlane(__shfl(j, 0)) * static_cast<int>(gridDim.x);
    };
    int t = t2 + static_cast<int>(blockIdx.x) + wv * static_cast<int>(gridDim.x);
    if (t >= n_tiles) {
#if NGNN_ROOT_TRACE
        if ((threadIdx.x & 63) == 0) atomicAdd(&g_root_trace[4], k1 - k0);
#endif
        return;
    }
    if (a.seed_dev) a.epi.drop.reseed(*a.seed_dev);
    const void *xbase = a.x_dev ? *a.x_dev : a.x;
    const i32x4 xr = make_rsrc_u(xbase, static_cast<uint32_t>((static_cast<int64_t>(n_rows - 1) * a.ldx + a.K) *
                                                             EB * (n_rows > 0)));
    const uint32_t ld4 = static_cast<uint32_t>(a.ldx) * EB;
    const int lane = threadIdx.x & 63, q = lane >> 4, rl = lane & 15;
#if NGNN_ROOT_TRACE
    unsigned long long tr[5] = {0, 0, 0, 0, k1 - k0};  // cycles: head+tail, root MFMAs, epilogue; tiles; prologue
#endif
    auto row_off = [&](int tt) __attribute__((always_inline)) -> uint32_t {
        const int rr = tt * RT_ROWS + rl;
        return rr < n_rows ? static_cast<uint32_t>(rr) * ld4 : static_cast<uint32_t>(kOOB);
    };
    // x fragments of a tile, X3 layout per 128-column group (load_x), and the
    // fp32 tail values (load_xt); rows past the block read 0
    auto load_tile = [&](v4f (&xf)[NXF], float (&xt)[T4N], uint32_t roff) __attribute__((always_inline)) {
#if NGNN_ROOT_NOLOAD  // (diagnostic: no x loads)
#pragma unroll
        for (int g = 0; g < NXF; ++g) xf[g] = v4f{float(roff), 1.f, 2.f, 3.f};
#pragma unroll
        for (int s2 = 0; s2 < T4N; ++s2) xt[s2] = float(roff);
        return;
#endif
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            if (XB) {
                const uint32_t voff = roff + static_cast<uint32_t>((128 * g + 8 * q) * 2);
#pragma unroll
                for (int c = 0; c < RT_KC / 2; ++c) {
                    xf[g * RT_KC + 2 * c] = (4 * g + c < CC) ? buf_load4(xr, static_cast<int>(voff + 64 * c), 0, 0)
                                                             : v4f{0.f, 0.f, 0.f, 0.f};
                    xf[g * RT_KC + 2 * c + 1] = v4f{0.f, 0.f, 0.f, 0.f};
                }
            } else {
                const uint32_t voff = roff + static_cast<uint32_t>((128 * g + 8 * q) * 4);
#pragma unroll
                for (int h = 0; h < RT_KC; ++h)
                    xf[g * RT_KC + h] = (4 * g + (h >> 1) < CC)
                                            ? buf_load4(xr, static_cast<int>(voff + 4 * (32 * (h >> 1) + 4 * (h & 1))), 0, 0)
                                            : v4f{0.f, 0.f, 0.f, 0.f};
            }
        }
        if constexpr (T4 > 0) {
#pragma unroll
            for (int s2 = 0; s2 < T4; ++s2) {
                const int e = 32 * CC + 4 * s2 + q;
                if (XB) {
                    const int w = buf_load1i(xr, static_cast<int>(roff + static_cast<uint32_t>((e & ~1) * 2)), 0, 0);
                    xt[s2] = __int_as_float((e & 1) ? (w & static_cast<int>(0xffff0000u)) : (w << 16));
                } else {
                    xt[s2] = buf_load1(xr, static_cast<int>(roff + static_cast<uint32_t>(e * 4)), 0, 0);
                }
            }
        }
    };

    // one tile on fragments (xc, xtc); the next tile's rows load into (xn, xtn)
    auto tile = [&](v4f (&xc)[NXF], const float (&xtc)[T4N], v4f (&xn)[NXF],
                    float (&xtn)[T4N]) __attribute__((always_inline)) -> bool {
        [[maybe_unused]] const unsigned long long c0 = rr_clock();
        const int tn = claim();
        load_tile(xn, xtn, row_off(tn));
        v4f acc[NTW];
#pragma unroll
        for (int m = 0; m < NTW; ++m) acc[m] = *reinterpret_cast<const v4f *>(sbias + 16 * m + 4 * q);
        if constexpr (T4 > 0) {
#pragma unroll
            for (int s2 = 0; s2 < T4; ++s2) {
                float wt[NTW];
#pragma unroll
                for (int m = 0; m < NTW; ++m) wt[m] = swt[(s2 * NTW + m) * 64 + lane];
                const float xv =
                    __int_as_float(__float_as_int(xtc[s2]) & lt_mask(32 * CC + 4 * s2 + q, a.K));
#pragma unroll
                for (int m = 0; m < NTW; ++m)
                    acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(wt[m], xv, acc[m], 0, 0, 0);
            }
        }
        [[maybe_unused]] const unsigned long long c1 = rr_clock();
        // W parts of step s = c NTW + m from a 3-slot ring, read two steps ahead
        bf16x8 wr[3][NP];
        auto load_w = [&](int s, bf16x8 (&w)[NP]) __attribute__((always_inline)) {
            const bf16x8 *p = sw3 + s * 64 + lane;
#pragma unroll
            for (int j = 0; j < NP; ++j) w[j] = p[j * pst];
        };
        load_w(0, wr[0]);
        if (NSTEP > 1) load_w(1, wr[1]);
#pragma unroll
        for (int c = 0; c < CC; ++c) {
            const int f = (c >> 2) * RT_KC + 2 * (c & 3);  // this chunk's fragments in xc
            bf16x8 x1, x2, x3;
            if constexpr (XB) {
                x1 = __builtin_bit_cast(bf16x8, xc[f]);
                x2 = x3 = x1;  // (unused)
            } else {
                split3<false>(xc[f], xc[f + 1], x1, x2, x3);
            }
#pragma unroll
            for (int m = 0; m < NTW; ++m) {
                const int s = c * NTW + m;
                if (s + 2 < NSTEP) load_w(s + 2, wr[(s + 2) % 3]);
                __builtin_amdgcn_sched_barrier(0);  // (keeps the ring's reads ahead)
                const bf16x8(&w)[NP] = wr[s % 3];
                v4f u = acc[m];
                if constexpr (W1 && XB) {
                    u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], x1, u, 0, 0, 0);
                } else if constexpr (W1) {
                    u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], x3, u, 0, 0, 0);
                    u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], x2, u, 0, 0, 0);
                    u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], x1, u, 0, 0, 0);
                } else if constexpr (XB) {
                    u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[NP - 1], x1, u, 0, 0, 0);
                    u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[NP - 2], x1, u, 0, 0, 0);
                    u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], x1, u, 0, 0, 0);
                } else {
                    u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[NP - 1], x1, u, 0, 0, 0);
                    u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], x3, u, 0, 0, 0);
                    u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[NP - 2], x2, u, 0, 0, 0);
                    u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[NP - 2], x1, u, 0, 0, 0);
                    u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], x2, u, 0, 0, 0);
                    u = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0], x1, u, 0, 0, 0);
                }
                acc[m] = u;
            }
        }
        [[maybe_unused]] const unsigned long long c2 = rr_clock();
        const i32x4 orsrc = OB ? tile_rsrc2(a.out, a.ldo, a.Fo, t, n_rows) : tile_rsrc(a.out, a.ldo, a.Fo, t, n_rows);
        const i32x4 zr = NAR ? tile_rsrc(a.z, a.ldz, 16 * a.NT1, t, n_rows) : orsrc;
        epilogue<NTW, DM, RELU, VEC, OB, NAR, false, NAR>(acc, a, orsrc, zr, t * RT_ROWS + rl, rl, q);
#if NGNN_ROOT_TRACE
        {
            // (acc consumed: the root MFMAs have drained before this point)
            const unsigned long long c3 = rr_clock();
            tr[0] += c1 - c0;
            tr[1] += c2 - c1;
            tr[2] += c3 - c2;
            tr[3] += 1;
        }
#endif
        t = tn;
        return t < n_tiles;
    };

    v4f xa[NXF], xb[NXF];
    float xta[T4N], xtb[T4N];
    load_tile(xa, xta, row_off(t));
    // settle the first tile's loads here: left pending on this entry path
    // (no stores behind them), the wait at the loop head would count no
    // younger stores on ANY path -- a drain of the previous tile's stores
    // every second tile
#pragma unroll
    for (int g = 0; g < NXF; ++g) asm volatile("" : "+v"(xa[g]));
#pragma unroll
    for (int s2 = 0; s2 < T4N; ++s2) asm volatile("" : "+v"(xta[s2]));
    while (tile(xa, xta, xb, xtb) && tile(xb, xtb, xa, xta)) {
    }
#if NGNN_ROOT_TRACE
    if ((threadIdx.x & 63) == 0)
        for (int i = 0; i < 5; ++i) atomicAdd(&g_root_trace[i], tr[i]);
#endif
}

template <int NTW, int CC, int T4, int FORM, bool XB, bool W1, bool VEC>
int go_root(const RtArgs &a, hipStream_t st) {
    auto fn = k_root<NTW, CC, T4, FORM, XB, W1, VEC>;
    constexpr int NP = W1 ? 1 : 3;
    const size_t lds = static_cast<size_t>(NP) * CC * NTW * 64 * 16 + static_cast<size_t>(T4) * NTW * 64 * 4 +
                       static_cast<size_t>(NTW) * 16 * 4;
    static bool attr_set = false;  // benign race: idempotent
    if (!attr_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(fn),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 256);
        attr_set = true;
    }
    const int64_t n_tiles = ceil_div(a.n_rows, RT_ROWS);
    const int grid = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(num_cus(), ceil_div(n_tiles, RR_WAVES))));
    hipLaunchKernelGGL(fn, dim3(grid), dim3(RR_WAVES * 64), lds, st, a);
    return launch_status();
}

}  // namespace

// The X3 root image of one slice in global memory, in the LDS layout
// (build_x3_image's), so each row-tile workgroup copies it instead of
// splitting W_r itself: that per-workgroup build -- scattered 32-B row reads
// from L2, split, LDS writes -- measured 12 us (layer 0) to 30 us (the narrow
// output layer) per launch.  One slot per thread.
template <int NTW, bool W1>
__global__ __launch_bounds__(256) void k_x3_image(RtArgs a, v4f *dst) {
    constexpr int NP = W1 ? 1 : 3;
    const int pst = a.C * NTW * 64;
    bf16x8 *sw3 = reinterpret_cast<bf16x8 *>(dst);
    float *swt = reinterpret_cast<float *>(dst + NP * pst);
    auto wrow = [&](int n) -> const float * {
        if (n >= 16 * a.NT) return nullptr;
        const bool zt = n >= 16 * a.NT1;
        const int nn = zt ? n - 16 * a.NT1 : n;
        const float *base = zt ? a.wz_raw : a.wr_raw;
        if (nn >= a.Fo || base == nullptr) return nullptr;
        return base + static_cast<int64_t>(nn) * a.ldw;
    };
    const int sl = blockIdx.x * 256 + threadIdx.x;
    if (sl < pst) {
        const int l = sl & 63, mt = (sl >> 6) % NTW, cc = (sl >> 6) / NTW;
        const int n = mt * 16 + (l & 15), k = 32 * cc + 8 * (l >> 4);
        v4f lo{0.f, 0.f, 0.f, 0.f}, hi{0.f, 0.f, 0.f, 0.f};
        const float *row = wrow(n);
        if (row) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                lo[j] = k + j < a.K ? row[k + j] : 0.0f;
                hi[j] = k + 4 + j < a.K ? row[k + 4 + j] : 0.0f;
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
    const int st = sl - pst;  // the fp32 tail slots
    if (st >= 0 && st < a.T4 * NTW * 64) {
        const int l = st & 63, mt = (st >> 6) % NTW, s2 = (st >> 6) / NTW;
        const int n = mt * 16 + (l & 15), k = 32 * a.C + 4 * s2 + (l >> 4);
        const float *row = wrow(n);
        swt[st] = (row && k < a.K) ? row[k] : 0.0f;
    }
    // the bf16 W_l image of the neighbour term (k_pack_wl_b16's layout), one
    // 16-B slot per thread past the root image's slots
    const int sb = st - a.T4 * NTW * 64;
    if (a.wlb_src && sb >= 0 && sb < ((a.wlb_fo + 15) >> 4) * a.CL * 64) {
        const int l = sb & 63, c = (sb >> 6) % a.CL, t = (sb >> 6) / a.CL;
        const int q = l >> 4, n = 16 * t + (l & 15);
        bf16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = 32 * c + (j < 4 ? 4 * q + j : 16 + 4 * q + j - 4);
            v[j] = static_cast<__bf16>((n < a.wlb_fo && k < a.K) ? a.wlb_src[static_cast<int64_t>(n) * a.ldw + k] : 0.0f);
        }
        reinterpret_cast<bf16x8 *>(const_cast<void *>(a.wlb))[sb] = v;
    }
    // the fp32 packed W_l (k_pack_weight's layout [NT][KG][64 lanes][4]: lane
    // l, element i of fragment (m, kg) holds W[16 m + (l & 15)][16 kg + 4 (l
    // >> 4) + i]), one fragment lane (4 floats) per thread past the above
    const int sp = sb - (a.wlb_src ? ((a.wlb_fo + 15) >> 4) * a.CL * 64 : 0);
    const int KG = (a.K + 15) >> 4;
    if (a.wlp_src && sp >= 0 && sp < ((a.wlp_fo + 15) >> 4) * KG * 64) {
        const int l = sp & 63, f = sp >> 6;
        const int n = 16 * (f / KG) + (l & 15), k = 16 * (f % KG) + 4 * (l >> 4);
        v4f v;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            v[j] = (n < a.wlp_fo && k + j < a.K) ? a.wlp_src[static_cast<int64_t>(n) * a.ldw + k + j] : 0.0f;
        a.wlp_dst[sp] = v;
    }
}

#if NGNN_ROOT_TRACE
extern "C" int ngnn_debug_root_trace(unsigned long long *out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_root_trace), sizeof(g_root_trace)) != hipSuccess) return -1;
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_root_trace), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

size_t x3_image_bytes(int ntw, int C, int T4, bool w1) {
    return static_cast<size_t>(w1 ? 1 : 3) * C * ntw * 64 * 16 + static_cast<size_t>(T4) * ntw * 64 * 4;
}

int build_image(RtArgs &a, int ntw, void *dst, hipStream_t st) {
    const int slots = a.C * ntw * 64 + a.T4 * ntw * 64 +
                      (a.wlb_src ? static_cast<int>(ceil_div(a.wlb_fo, 16)) * a.CL * 64 : 0) +
                      (a.wlp_src ? static_cast<int>(ceil_div(a.wlp_fo, 16) * ceil_div(a.K, 16)) * 64 : 0);
    const unsigned grid = static_cast<unsigned>(ceil_div(slots, 256));
    v4f *d = static_cast<v4f *>(dst);
    const bool w1 = a.w1 != 0;
#define NGNN_IMG(N)                                                                           \
    if (ntw == N) {                                                                           \
        if (w1) hipLaunchKernelGGL((k_x3_image<N, true>), dim3(grid), dim3(256), 0, st, a, d);  \
        else hipLaunchKernelGGL((k_x3_image<N, false>), dim3(grid), dim3(256), 0, st, a, d);    \
    }
    NGNN_IMG(2) NGNN_IMG(3) NGNN_IMG(4) NGNN_IMG(6) NGNN_IMG(8) NGNN_IMG(16)
#undef NGNN_IMG
    const int rc = launch_status();
    if (rc) return rc;
    a.img = d;
    return NGNN_OK;
}

int rt_form(const RtArgs &a, int ntw, bool vec) {
    if (a.NT1 < a.NT) return (a.NT == ntw && 2 * a.NT1 == ntw && a.epi.drop.thresh == 0u && !a.epi.relu) ? 4 : 0;
    if ((a.epi.col_base >> 4) & 1) return 0;  // (odd column slices: the hash word parity)
    int f = 0;
    if (a.epi.drop.thresh == 128u && a.epi.relu) f = 1;
    else if (a.epi.drop.thresh == 0u && a.epi.relu) f = 2;
    else if (a.epi.drop.thresh == 0u && !a.epi.relu) f = 3;
    if (f && a.out_bf16) f = (f == 3 || !vec || !a.w1) ? 0 : f + 4;
    return f;
}

// The instantiated shapes: the benched configs' layers (fp32: products /
// arxiv layer 0 and the narrow output layer; bf16 models: layer 0, the
// 256 -> 256 hidden layer and the narrow output layer).  Everything else
// keeps k_sage_rt's own root-term loop.
int launch_root(const RtArgs &a, int ntw, int form, bool vec, hipStream_t st, bool dry) {
    if (a.kpad || a.xrow || a.xrow_dev || !a.wr_raw) return NGNN_E_SHAPE;
    const bool xb = a.x_bf16 != 0, w1 = a.w1 != 0;
    const int C = a.C, T4 = a.T4;
#define NGNN_ROOT(NTW_, CC_, T4_, F_, XB_, W1_, VEC_)                                                   \
    if (ntw == NTW_ && C == CC_ && T4 == T4_ && form == F_ && xb == XB_ && w1 == W1_ && vec == VEC_) \
        return dry ? NGNN_OK : go_root<NTW_, CC_, T4_, F_, XB_, W1_, VEC_>(a, st);
    // fp32 layer 0: products K = 100 (3 chunks + a 4-column tail), arxiv K = 128
    NGNN_ROOT(16, 3, 1, 1, false, false, true)
    NGNN_ROOT(16, 3, 1, 2, false, false, true)
    NGNN_ROOT(16, 3, 1, 3, false, false, true)
    NGNN_ROOT(16, 4, 0, 1, false, false, true)
    NGNN_ROOT(16, 4, 0, 2, false, false, true)
    NGNN_ROOT(16, 4, 0, 3, false, false, true)
    // narrow output layer 256 -> 47 / 40 (out and z, 3 + 3 tiles), fp32 and bf16 rows
    NGNN_ROOT(6, 8, 0, 4, false, false, false)
    NGNN_ROOT(6, 8, 0, 4, true, true, false)
    // bf16 models: layer 0 (bf16 rows, K = 100) and the 256 -> 256 hidden layer, bf16 out
    NGNN_ROOT(16, 3, 1, 5, true, true, true)
    NGNN_ROOT(16, 3, 1, 6, true, true, true)
    NGNN_ROOT(16, 8, 0, 5, true, true, true)
    NGNN_ROOT(16, 8, 0, 6, true, true, true)
#undef NGNN_ROOT
    return NGNN_E_SHAPE;
}

}  // namespace ngnn
