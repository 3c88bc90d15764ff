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

#include "ngnn_sage_rt_kern.h"

namespace ngnn {
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

namespace {

// (NTW, reduce) -> the instantiation unit's entry (ngnn_rt_tu.hip)
int dispatch_rt(int ntw, const RtArgs &a, int reduce, bool wl_lds, bool x3, int n_tiles,
                size_t lds, hipStream_t st) {
#define NGNN_RT_CALL(N, R) \
    if (ntw == N && reduce == R) return NGNN_RT_FN(N, R)(a, wl_lds, x3, n_tiles, lds, st);
    NGNN_RT_FOR_EACH(NGNN_RT_CALL)
#undef NGNN_RT_CALL
    return NGNN_E_ARG;
}

// ---- narrow-mode neighbour term: out[d, :Fo] += reduce_{e into d} z[col[e], :Fo]
// for rows d with in-edges below min(n_rows, *n_rows_dev, *n_edge_rows_dev):
// mean/sum of z = x W_l^T (linear, so equal to W_l . mean(x) up to fp32
// rounding).  16 lanes per row (float4 columns), 4 rows per wave, 8
// neighbour rows in flight per lane; per column edge order from 0, then
// / deg for mean.
constexpr int NA_UNR = 16;

// max / sum over the 16 lanes of a row group (a DPP row: lanes 16 k ..
// 16 k + 15, all active together) on VALU only: quad_perm [1,0,3,2] and
// [2,3,0,1] combine a quad, row_half_mirror the two quads of a half,
// row_mirror the two halves -- every lane ends with the row's value
__device__ __forceinline__ float max16(float v) {
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false)));
    return fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false)));
}
__device__ __forceinline__ float sum16(float v) {
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
}

// HEAD (the loss head, ngnn_xent_head): the rows d < B are visited with or
// without in-edges; once a row's logits are final the group takes its cross
// entropy -- max, sum of exp and the label's logit over the group, the
// gradient row (softmax - onehot) / count as ngnn_seed_xent_fwd_grad writes
// it -- and scatters the gradient row onto its sources (g[col[e]] += dy[d] /
// deg(d), as the backward's narrow scatter).  count: every workgroup that
// holds seed rows counts the valid labels itself (B label reads from L2, no
// count pass).  The loss: per-group sums in row order, per workgroup in
// group order, and the last workgroup to finish (a device ticket) adds the
// workgroup partials in a fixed order -- deterministic; the hand-off is
// k_xent_fused's (ngnn_loss.hip: agent-scope partial stores drained before
// one ticket atomic, agent-scope loads by the last adder).
// WIDE: z row offsets by a full 32-bit multiply (n_rows or the row bytes past
// 24 bits); else v_mul_u32_u24.  Edge offsets are unsigned 32-bit: col reads
// are exact below 2^30 edges (the resource's 3.75 GiB range).
template <bool MEAN, bool HEAD, bool WIDE = false>
__global__ __launch_bounds__(256) void k_narrow_agg(const float *__restrict__ z, int64_t ldz, int Fo,
                                                    const int32_t *__restrict__ rowptr,
                                                    const int32_t *__restrict__ col, int n_rows,
                                                    const int32_t *__restrict__ n_rows_dev,
                                                    const int32_t *__restrict__ n_edge_dev,
                                                    float *__restrict__ out, int64_t ldo, NarrowHead hd) {
    int nr = n_rows;
    if (n_rows_dev) nr = min(nr, *n_rows_dev);
    if (n_edge_dev) nr = min(nr, *n_edge_dev);
    const int sub = threadIdx.x & 15;
    const int F4 = (Fo + 3) >> 2;
    // index words through buffer resources (masked slots read 0, no
    // branches): a row's first 16 neighbour ids in ONE round trip, then its
    // 16 z rows in one more (a fanout of <= 16 needs exactly two)
    const i32x4 cr = make_rsrc(col, 0xF0000000u);
    const uint32_t ldz4 = static_cast<uint32_t>(ldz) * 4u;
    constexpr int OOB = static_cast<int>(0xF0000000u);
    // the neighbour mean / sum of z of row d, columns 4 c4 .. 4 c4 + 3
    auto gather = [&](int beg, int end, int c4) __attribute__((always_inline)) {
        v4f acc{0.f, 0.f, 0.f, 0.f};
        for (int e = beg; e < end; e += NA_UNR) {
            int id[NA_UNR];
#pragma unroll
            for (int u = 0; u < NA_UNR; ++u)
                id[u] = buf_load1i(cr, e + u < end ? static_cast<int>(4u * static_cast<uint32_t>(e + u)) : OOB, 0, 0);
            const i32x4 zr = make_rsrc(z, 0xF0000000u);
            v4f v[NA_UNR];
#pragma unroll
            for (int u = 0; u < NA_UNR; ++u)
                v[u] = buf_load4(zr, e + u < end ? static_cast<int>((WIDE ? static_cast<uint32_t>(id[u]) * ldz4
                                                               : __umul24(static_cast<uint32_t>(id[u]), ldz4))) + 16 * c4
                                                  : OOB,
                                 0, 0);
#pragma unroll
            for (int u = 0; u < NA_UNR; ++u)
                if (e + u < end) acc += v[u];
        }
        if (MEAN && end > beg) acc = acc / static_cast<float>(end - beg);
        return acc;
    };
    const int stride = (gridDim.x * blockDim.x) >> 4;
    if constexpr (!HEAD) {
        for (int d = (blockIdx.x * blockDim.x + threadIdx.x) >> 4; d < nr; d += stride) {
            const int beg = rowptr[d], end = rowptr[d + 1];
            if (beg == end) continue;
            for (int c4 = sub; c4 < F4; c4 += 16) {
                const v4f acc = gather(beg, end, c4);
                float *o = out + static_cast<int64_t>(d) * ldo + 4 * c4;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (4 * c4 + j < Fo) o[j] += acc[j];
            }
        }
    } else {
        // (host: F4 <= 16, one column quad per lane; B <= n_rows)
        __shared__ float s_red[256];
        __shared__ float s_grp[16];
        // rows to workgroups as the plain kernel's (16 consecutive row slots
        // per workgroup and pass), except that the first 2 B8 slots (B8 =
        // ceil8(B)) interleave: a workgroup's groups 0-7 take 8 consecutive
        // seed rows, groups 8-15 the 8 rows B8 + the same offset -- the seed
        // rows, and their scatter atomics, spread over twice the workgroups
        // with the row locality kept.  (Measured alternatives,
        // tools/fwd2_micro.py --head: seed rows one per workgroup over all
        // of them spread the atomics but cost the rest of the launch its row
        // locality, 36 us against 18; 4 per workgroup on wave 0 of ceil(B /
        // 4) workgroups, 25.)
        const int B = hd.B, G = static_cast<int>(gridDim.x), bx = static_cast<int>(blockIdx.x);
        const int B8 = (B + 7) & ~7;
        const int nh = min(G, B8 >> 3);  // workgroups holding seed rows
        const bool hwg = bx < nh;              // (uniform)
        float cnt = 0.0f;
        if (hd.cnt_in) {
            cnt = *hd.cnt_in;
        } else if (hwg) {
            float c = 0.0f;
            for (int i = threadIdx.x; i < B; i += 256) c += (hd.y[i] != hd.ignore) ? 1.0f : 0.0f;
            s_red[threadIdx.x] = c;
            __syncthreads();
            for (int h = 128; h > 0; h >>= 1) {
                if (threadIdx.x < h) s_red[threadIdx.x] += s_red[threadIdx.x + h];
                __syncthreads();
            }
            cnt = s_red[0];
        }
        float lsum = 0.0f;
        const int c4 = sub;
        const i32x4 zr = make_rsrc(z, 0xF0000000u);
        // the seed-edge counts of this call (the selector read once; the
        // loss's last adder flips it below, after every head workgroup read it)
        int ssel = 0;
        i32x4 scr = make_rsrc(nullptr, 0u);
        if (hd.scnt_base && hwg) {
            ssel = hd.scnt_base[2 * hd.scnt_stride] & 1;
            scr = make_rsrc(hd.scnt_base + ssel * hd.scnt_stride, static_cast<uint32_t>(hd.scnt_stride) * 4u);
        }
        const int dl = max(nr, B);
        const int vl = max(dl, 2 * B8);
        for (int v = (bx * 256 + static_cast<int>(threadIdx.x)) >> 4; v < vl; v += 16 * G) {
            const int vg = v & 15;
            const int d = v < 2 * B8 ? ((v >> 4) << 3) + (vg & 7) + (vg >= 8 ? B8 : 0) : v;
            if (d >= dl) continue;
            const bool hrow = d < B;
            const int beg = rowptr[d], end = (d < nr) ? rowptr[d + 1] : beg;
            if (beg == end && !hrow) continue;
            // the label, the root logits and the first 16 neighbour ids in
            // one round trip; the ids stay in registers for the scatter
            const int64_t t = hrow ? hd.y[d] : 0;
            float *o = out + static_cast<int64_t>(d) * ldo + 4 * c4;
            v4f ov{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (4 * c4 + j < Fo) ov[j] = o[j];
            int id[NA_UNR];
#pragma unroll
            for (int u = 0; u < NA_UNR; ++u) id[u] = buf_load1i(cr, beg + u < end ? 4 * (beg + u) : OOB, 0, 0);
            v4f acc{0.f, 0.f, 0.f, 0.f};
            // a seed row's sources' edge counts (1: the source's g row takes
            // one plain store); read with the gathers, used at the scatter
            int scn[NA_UNR];
#pragma unroll
            for (int u = 0; u < NA_UNR; ++u)
                scn[u] = buf_load1i(scr, (hrow && beg + u < end) ? static_cast<int>(4u * static_cast<uint32_t>(id[u])) : OOB, 0, 0);
            if (c4 < F4 && end > beg) {
                v4f v[NA_UNR];
#pragma unroll
                for (int u = 0; u < NA_UNR; ++u)
                    v[u] = buf_load4(zr, beg + u < end ? static_cast<int>(__umul24(static_cast<uint32_t>(id[u]), ldz4)) + 16 * c4 : OOB,
                                     0, 0);
#pragma unroll
                for (int u = 0; u < NA_UNR; ++u)
                    if (beg + u < end) acc += v[u];
                // (rare: more than 16 neighbours -- the rest in further round trips,
                // edge order kept: the sum continues from the first 16)
                for (int e = beg + NA_UNR; e < end; e += NA_UNR) {
                    int ie[NA_UNR];
#pragma unroll
                    for (int u = 0; u < NA_UNR; ++u) ie[u] = buf_load1i(cr, e + u < end ? 4 * (e + u) : OOB, 0, 0);
#pragma unroll
                    for (int u = 0; u < NA_UNR; ++u)
                        v[u] = buf_load4(zr, e + u < end ? static_cast<int>(__umul24(static_cast<uint32_t>(ie[u]), ldz4)) + 16 * c4 : OOB,
                                         0, 0);
#pragma unroll
                    for (int u = 0; u < NA_UNR; ++u)
                        if (e + u < end) acc += v[u];
                }
                if (MEAN) acc = acc / static_cast<float>(end - beg);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (4 * c4 + j < Fo && end > beg) {
                    ov[j] = ov[j] + acc[j];
                    o[j] = ov[j];  // (edgeless rows keep their bits, -0.0 included)
                }
            if (!hrow) continue;
            if (hd.dbg & 4) continue;  // (profiling: no cross entropy)
            // the row's cross entropy (torch's log_softmax order: max, then
            // the sum of exp(x - max))
            float m = -INFINITY;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (4 * c4 + j < Fo) m = fmaxf(m, ov[j]);
            m = max16(m);
            float s = 0.0f, ot = 0.0f;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (4 * c4 + j < Fo) {
                    s += expf(ov[j] - m);
                    if (4 * c4 + j == t) ot = ov[j];
                }
            s = sum16(s);
            ot = sum16(ot);  // (the label's logit: one lane holds it, the others add 0)
            const float lse = m + logf(s);
            const bool ign = t == hd.ignore;
            const float l = ign ? 0.0f : ((t >= 0 && t < Fo) ? lse - ot : NAN);  // out-of-range label: NaN
            v4f dv{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (4 * c4 + j < Fo && !ign) dv[j] = (expf(ov[j] - lse) - (4 * c4 + j == t ? 1.0f : 0.0f)) / cnt;
            float *dr = hd.dy + static_cast<int64_t>(d) * hd.ldd + 4 * c4;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (4 * c4 + j < Fo) dr[j] = dv[j];
            if (hd.g && !ign && end > beg && !(hd.dbg & 1)) {
                if (MEAN) dv = dv * (1.0f / static_cast<float>(end - beg));
                // the row's sources from the registers (no load between the
                // atomics); past 16 neighbours, reloaded 16 at a time
#pragma unroll
                for (int u = 0; u < NA_UNR; ++u)
                    if (beg + u < end) {
                        float *gr = hd.g + static_cast<int64_t>(id[u]) * hd.ldg + 4 * c4;
                        if (scn[u] == 1) {
                            // the source's only seed edge: its g row (zeroed by
                            // the edge launch) is this row's contribution
                            if (c4 < F4) *reinterpret_cast<v4f *>(gr) = dv;
                        } else {
#pragma unroll
                            for (int j = 0; j < 4; ++j)
                                if (4 * c4 + j < Fo && dv[j] != 0.0f) atomicAdd(gr + j, dv[j]);  // exact 0 adds nothing
                        }
                    }
                for (int e = beg + NA_UNR; e < end; e += NA_UNR) {
                    int ie[NA_UNR];
#pragma unroll
                    for (int u = 0; u < NA_UNR; ++u) ie[u] = buf_load1i(cr, e + u < end ? 4 * (e + u) : OOB, 0, 0);
#pragma unroll
                    for (int u = 0; u < NA_UNR; ++u)
                        if (e + u < end) {
                            float *gr = hd.g + static_cast<int64_t>(ie[u]) * hd.ldg + 4 * c4;
#pragma unroll
                            for (int j = 0; j < 4; ++j)
                                if (4 * c4 + j < Fo && dv[j] != 0.0f) atomicAdd(gr + j, dv[j]);
                        }
                }
            }
            lsum += l;
        }
        if (hwg && !(hd.dbg & 2)) {
            // the loss: the workgroup's rows in group order, then a two-level
            // hand-off by one lane behind an LDS-only barrier (the waves'
            // scatter atomics and stores stay in flight) -- groups of 32
            // workgroups count on their own ticket, the last of a group adds
            // the group's partials in order and counts on the top ticket,
            // whose last adds the group sums in order (same-address atomics
            // serialise at the memory side: 32 per address instead of one per
            // workgroup)
            if (sub == 0) s_grp[threadIdx.x >> 4] = lsum;
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            float p = 0.0f;
            for (int i = 0; i < 16; ++i) p += s_grp[i];
            if (threadIdx.x == 0) {
                float *gpart = hd.part;            // [32] group sums
                float *wpart = hd.part + 32;       // [nh] workgroup partials
                uint32_t *tick1 = hd.ticket + 16;  // [32] group tickets
                __hip_atomic_store(wpart + bx, p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const int gi = bx >> 5, g0 = gi << 5, gs = min(32, nh - g0), ngr = (nh + 31) >> 5;
                if (atomicAdd(tick1 + gi, 1u) == static_cast<uint32_t>(gs - 1)) {
                    float v[32];
#pragma unroll
                    for (int i = 0; i < 32; ++i)
                        v[i] = i < gs ? __hip_atomic_load(wpart + g0 + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0f;
                    float a = 0.0f;
#pragma unroll
                    for (int i = 0; i < 32; ++i) a += v[i];
                    tick1[gi] = 0u;  // (every member has counted: ready for the next call)
                    __hip_atomic_store(gpart + gi, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if (atomicAdd(hd.ticket, 1u) == static_cast<uint32_t>(ngr - 1)) {
#pragma unroll
                        for (int i = 0; i < 32; ++i)
                            v[i] = i < ngr ? __hip_atomic_load(gpart + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0f;
                        float t = 0.0f;
#pragma unroll
                        for (int i = 0; i < 32; ++i) t += v[i];
                        *hd.loss = t / cnt;  // 0/0 = NaN when every row is ignored, as torch
                        *hd.count = cnt;
                        *hd.ticket = 0u;
                        // the next call's edge launch counts into the other array
                        if (hd.scnt_base) hd.scnt_base[2 * hd.scnt_stride] = ssel ^ 1;
                    }
                }
            }
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

// W_l [Fo, K] (bf16-exact fp32 values, row stride ldw) -> the bf16 image
// [NT][CL][64] x 8 of the row-tile kernel's bf16 neighbour term (RtArgs::wlb):
// element j of lane (q, m) in chunk c is W_l[16 t + m][32 c + 4 q + j] (j < 4)
// or [32 c + 16 + 4 q + j - 4] (j >= 4); zero outside Fo x K.  One thread per
// element (RNE conversion -- exact on bf16-exact weights).
__global__ __launch_bounds__(256) void k_pack_wl_b16(const float *__restrict__ w, int64_t ldw, int Fo, int K,
                                                     int CL, int NT, uint16_t *__restrict__ dst) {
    const int64_t idx = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
    if (idx >= static_cast<int64_t>(NT) * CL * 512) return;
    const int j = idx & 7, lane = (idx >> 3) & 63;
    const int64_t tc = idx >> 9;
    const int c = static_cast<int>(tc % CL), t = static_cast<int>(tc / CL);
    const int q = lane >> 4, n = 16 * t + (lane & 15);
    const int k = 32 * c + (j < 4 ? 4 * q + j : 16 + 4 * q + j - 4);
    const float v = (n < Fo && k < K) ? w[static_cast<int64_t>(n) * ldw + k] : 0.0f;
    dst[idx] = __builtin_bit_cast(uint16_t, static_cast<__bf16>(v));
}

}  // namespace

// bytes of the bf16 W_l image (k_pack_wl_b16)
size_t wl_b16_bytes(int64_t Fo, int64_t K) {
    return static_cast<size_t>(ceil_div(Fo, 16)) * static_cast<size_t>(ceil_div(K, 32)) * 64 * 16;
}

// out[d, :Fo] += mean / sum_{e into d} z[col[e], :Fo] for the rows with
// in-edges (the narrow output layer's neighbour term; also ngnn_fwd2.hip);
// head (nullable): the loss head over rows < head->B (ngnn_fwd2.hip)
int narrow_agg_launch(const float *z, int64_t ldz, int64_t Fo, const int32_t *rowptr, const int32_t *col,
                      int64_t n_rows, const int32_t *n_rows_dev, int64_t n_edge_rows,
                      const int32_t *n_edge_rows_dev, int reduce, float *out, int64_t ldo, hipStream_t st,
                      const NarrowHead *head) {
    const int64_t rows = std::max<int64_t>(1, std::min(n_edge_rows, n_rows));
    // (32-bit buffer offsets into z; past 24-bit rows or row bytes the z
    // offsets take the full multiply: k_narrow_agg<..., WIDE>)
    NGNN_RETURN_IF(n_rows * ldz * 4 >= 0xF0000000ll, NGNN_E_RANGE);
    const bool wide = n_rows >= (1 << 24) || ldz * 4 >= (1 << 24);
    NGNN_RETURN_IF(head && (Fo > 64 || head->B <= 0 || head->B > n_rows), NGNN_E_ARG);
    NGNN_RETURN_IF(head && n_rows >= (1 << 24), NGNN_E_RANGE);
    const unsigned grid = static_cast<unsigned>(
        std::max<int64_t>(1, std::min<int64_t>(head ? std::min(4 * num_cus(), 1024) : 4 * num_cus(),
                                               ceil_div(std::max<int64_t>(rows, head ? 2 * ((head->B + 7) & ~int64_t{7}) : 0), 16))));
    // (the head's hand-off: at most 32 groups of 32 workgroups)
    const NarrowHead hd = head ? *head : NarrowHead{};
    auto go = [&](auto mean_c, auto head_c) {
        if (wide && !decltype(head_c)::value)  // (the loss head's blocks are NeighborLoader-sized)
            hipLaunchKernelGGL((k_narrow_agg<decltype(mean_c)::value, false, true>), dim3(grid), dim3(256), 0,
                               st, z, ldz, static_cast<int>(Fo), rowptr, col, static_cast<int>(n_rows), n_rows_dev,
                               n_edge_rows_dev, out, ldo, hd);
        else
            hipLaunchKernelGGL((k_narrow_agg<decltype(mean_c)::value, decltype(head_c)::value>), dim3(grid), dim3(256),
                               0, st, z, ldz, static_cast<int>(Fo), rowptr, col, static_cast<int>(n_rows), n_rows_dev,
                               n_edge_rows_dev, out, ldo, hd);
    };
    const bool mean = reduce == NGNN_REDUCE_MEAN;
    if (head) {
        if (mean) go(std::true_type{}, std::true_type{});
        else go(std::false_type{}, std::true_type{});
    } else {
        if (mean) go(std::true_type{}, std::false_type{});
        else go(std::false_type{}, std::false_type{});
    }
    return launch_status();
}

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
                     const int32_t *col_x, bool x_bf16, bool w_bf16, bool wl_prepacked,
                     bool agg_pre, bool out_bf16, int64_t n_edge_rows,
                     const int32_t *n_edge_rows_dev, void *img_ws) {
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
    if (x_bf16 && (!x3 || ldx % 4 != 0)) return 0;
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
        // (the root image's launch packs the weights below when that image
        // is prebuilt)
        const bool img_pre = x3 && !no_root && img_ws && x3_image_bytes(NTW, C, T4, w1) <= kImgWsBytes;
        a.wlp_src = nullptr;
        a.wlp_dst = nullptr;
        a.wlp_fo = 0;
        if (ldw && has_l && !wl_lds) {
            // raw W_l that must stream from L2: pack it once (all slices) into
            // the caller's workspace -- fragment-ordered 1-KiB wave loads
            // (one-part layers stream the bf16 image below instead: no fp32 pack)
            if (c0 == 0 && !w1) {
                if (!wl_ws || wl_ws_bytes < ngnn_pack_weight_bytes(Fo, K)) {
                    *rc = NGNN_E_WORKSPACE;
                    return 1;
                }
                // (NGNN_WL_PREPACKED: the producer packed this step's W_l there;
                // with a prebuilt root image its launch packs it: one launch)
                if (!wl_prepacked && img_pre) {
                    a.wlp_src = static_cast<const float *>(wl_packed);
                    a.wlp_dst = static_cast<v4f *>(wl_ws);
                    a.wlp_fo = static_cast<int>(Fo);
                }
                const int prc = (wl_prepacked || img_pre) ? 0
                                                          : ngnn_pack_weight(static_cast<const float *>(wl_packed),
                                                                             ldw, Fo, K, wl_ws, st);
                if (prc) {
                    *rc = prc;
                    return 1;
                }
            }
            a.wl = static_cast<const v4f *>(wl_ws) + toff;
        }
        // one-part (bf16-exact) W_l streamed from L2: the neighbour term on
        // bf16 MFMA from a bf16 image behind the packed fp32 one in the
        // workspace (the kernel's W1 streamed form has no fp32 steps)
        a.wlb = nullptr;
        a.wlb_src = nullptr;
        a.wlb_fo = static_cast<int>(Fo);
        a.CL = static_cast<int>(ceil_div(K, 32));
        if (w1 && has_l && !wl_lds) {
            if (!ldw || !wl_ws || wl_ws_bytes < ngnn_pack_weight_bytes(Fo, K) + wl_b16_bytes(Fo, K)) {
                *rc = NGNN_E_WORKSPACE;
                return 1;
            }
            uint16_t *img16 = reinterpret_cast<uint16_t *>(static_cast<char *>(wl_ws) + ngnn_pack_weight_bytes(Fo, K));
            if (c0 == 0 && img_pre) {
                a.wlb = img16;
                a.wlb_src = static_cast<const float *>(wl_packed);
            } else if (c0 == 0) {
                const int NTa = static_cast<int>(ceil_div(Fo, 16));
                const int64_t total = static_cast<int64_t>(NTa) * a.CL * 512;
                hipLaunchKernelGGL(k_pack_wl_b16, dim3(static_cast<unsigned>(ceil_div(total, 256))), dim3(256), 0, st,
                                   static_cast<const float *>(wl_packed), ldw, static_cast<int>(Fo),
                                   static_cast<int>(K), a.CL, NTa, img16);
                *rc = launch_status();
                if (*rc) return 1;
            }
            a.wlb = img16 + (c0 / 16) * a.CL * 64 * 8;
        }
        a.NT = NT;
        a.NT1 = NT1;
        // (unknown: every row may have in-edges -- no root-only phase)
        a.n_edge = static_cast<int>(n_edge_rows < 0 ? n_rows : std::min(n_edge_rows, n_rows));
        a.n_edge_dev = n_edge_rows_dev;
        a.root_split = 0;
        a.wz_raw = narrow ? static_cast<const float *>(wl_packed) : nullptr;
        a.z = z;
        a.ldz = ldz;
        a.Fo = static_cast<int>(Fo_c);
        a.out = out_bf16 ? reinterpret_cast<float *>(reinterpret_cast<uint16_t *>(out) + c0) : out + c0;
        a.ldo = ldo;
        a.vec_out = (Fo_c % 4 == 0) && (ldo % 4 == 0) && aligned(a.out, out_bf16 ? 8 : 16);
        a.out_bf16 = out_bf16;
        if (out_bf16 && !(a.vec_out && Fo_c % 16 == 0 && w1)) {  // bf16 rows: whole 16-column tiles of a one-part-image layer
            *rc = NGNN_E_SHAPE;
            return 1;
        }
        a.agg_out = (c0 == 0 && !narrow && !agg_pre) ? agg_out : nullptr;
        a.ld_agg = ld_agg;
        // later column slices read the aggregate the first one saved (the
        // launches are stream-ordered) instead of gathering it again; agg_pre:
        // every slice reads it (written by a separate aggregate launch)
        a.agg_in = ((c0 > 0 || agg_pre) && !narrow && has_l) ? agg_out : nullptr;
        a.epi = Epi{bias ? bias + c0 : nullptr, relu, drop, static_cast<int>(c0)};
        a.seed_dev = seed_dev;
        a.x_dev = x_dev;
        a.xrow = xrow;
        a.xrow_dev = xrow_dev;
        a.x_rows = x_rows;
        a.col_x = (xrow || xrow_dev) ? col_x : nullptr;
        a.x_bf16 = x_bf16;
        a.w1 = w1;
        // the split-bf16 root image built once (k_x3_image) into img_ws and
        // DMA-copied by every workgroup (else each workgroup builds it)
        a.img = nullptr;
        if (img_pre) {
            *rc = build_image(a, NTW, img_ws, st);
            if (*rc) return 1;
        }
        a.wlb_src = nullptr;
        a.wlp_src = nullptr;
        const int n_tiles = static_cast<int>(ceil_div(n_rows, RT_ROWS));
        // the tiles past the edge-row bound on k_root (ngnn_root.hip) when an
        // instantiation covers this layer: k_sage_rt takes the tiles with
        // in-edges (none in narrow mode), then k_root the rest
        const bool vec = a.vec_out && (a.Fo == a.NT * 16);
        const int form = (x3 && !NGNN_RT_STATIC && !no_root) ? rt_form(a, NTW, vec) : 0;
        // policy (NGNN_ROOT, read once): 1 (default) k_root for layers with no
        // in-kernel neighbour term (narrow mode: every tile); 2 also split the
        // layers with edge tiles (k_sage_rt edge tiles, then k_root -- measured
        // slower on products layer 0: the edge tiles alone then hold the GPU
        // ~48 us, in one launch they overlap the root tiles); 0 never
        static const int policy = [] {
            const char *e = std::getenv("NGNN_ROOT");
            return e ? std::atoi(e) : 1;
        }();
        const bool want_root = policy == 2 || (policy == 1 && !a.wl);
        if (form && want_root && launch_root(a, NTW, form, vec, st, true) == NGNN_OK) {
            if (a.wl) {
                a.root_split = 1;
                *rc = dispatch_rt(NTW, a, reduce, wl_lds, x3, n_tiles, lds, st);
                if (*rc) return 1;
                a.root_split = 0;
            }
            *rc = launch_root(a, NTW, form, vec, st);
            if (*rc) return 1;
            continue;
        }
        *rc = dispatch_rt(NTW, a, reduce, wl_lds, x3, n_tiles, lds, st);
        if (*rc) return 1;
    }
    return 1;
}

}  // namespace ngnn

using namespace ngnn;

extern "C" size_t ngnn_sage_fwd_raw_workspace_bytes(int64_t K, int64_t Fo, int64_t n_rows) {
    // a packed W_l (when it cannot sit in LDS), or narrow mode's z rows, or
    // the wide path's aggregate rows (inference: no saved-aggregate buffer)
    const size_t z = static_cast<size_t>(std::max<int64_t>(n_rows, 0)) * ceil_div(Fo, 16) * 16 *
                     sizeof(float);
    // (the wide tail: X3's 6-part weight image, or H2's 2-part image + its
    // row / column exponent arrays -- whichever is larger for these rows, so
    // the H2 form never drops back to X3 for want of room)
    const size_t nr = static_cast<size_t>(std::max<int64_t>(n_rows, 0));
    const size_t h2_tail = static_cast<size_t>(8) * Fo * ceil_div(K, 32) * 32 + (2 * Fo + 2 * nr) * 4 + 1024 + 512;
    const size_t wide = (sage_wide_preferred(K, Fo, false) || sage_wide_preferred(K, Fo, true))
                            ? sage_wide_workspace_bytes(K, n_rows) + std::max(wide_wimg_bytes(K, Fo), h2_tail) + 256
                            : 0;
    // + the prebuilt root image at the workspace's tail (kImgWsBytes); the
    // packed W_l is followed by its bf16 image (one-part layers)
    return std::max({ngnn_pack_weight_bytes(Fo, K) + wl_b16_bytes(Fo, K), z, wide}) + kImgWsBytes;
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
    const bool exact = (reduce & NGNN_MATH_EXACT_F32) != 0;
    const bool want_narrow = (reduce & NGNN_FWD_NARROW) != 0;
    const bool x_bf16 = (reduce & NGNN_X_BF16) != 0;
    const bool w_bf16 = (reduce & NGNN_W_BF16) != 0;
    const bool wl_prepacked = (reduce & NGNN_WL_PREPACKED) != 0;
    const bool out_bf16 = (reduce & NGNN_OUT_BF16) != 0;
    reduce &= ~(NGNN_MATH_EXACT_F32 | NGNN_FWD_NARROW | NGNN_X_BF16 | NGNN_W_BF16 |
                NGNN_WL_PREPACKED | NGNN_OUT_BF16);
    // bf16 rows: the split-bf16 root term only
    if (x_bf16 && exact) return NGNN_E_SHAPE;
    if (out_bf16 && want_narrow) return NGNN_E_SHAPE;
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
    // the root image's region: the workspace's last kImgWsBytes (16-B aligned)
    // when the rest still holds z (narrow) / a packed W_l
    const size_t head = want_narrow ? static_cast<size_t>(n_rows) * ldz * sizeof(float)
                                    : ngnn_pack_weight_bytes(Fo, K) + wl_b16_bytes(Fo, K);
    void *img_ws = nullptr;
    // (NGNN_IMG=0, read once: every workgroup builds its image -- A/B only)
    static const bool img_on = [] {
        const char *e = std::getenv("NGNN_IMG");
        return !e || std::atoi(e) != 0;
    }();
    if (img_on && ws && aligned(ws, 16) && ws_bytes >= head + kImgWsBytes + 16) {
        const uintptr_t e = (reinterpret_cast<uintptr_t>(ws) + ws_bytes - kImgWsBytes) & ~uintptr_t(15);
        img_ws = reinterpret_cast<void *>(e);
    }
    if (want_narrow && wl && reduce != NGNN_REDUCE_MAX && !agg_out && !relu && !(p_drop > 0.0f) &&
        ws && aligned(ws, 16) &&
        ws_bytes >= static_cast<size_t>(n_rows) * ldz * sizeof(float)) {
        float *z = static_cast<float *>(ws);
        if (sage_fwd_rowtile(x, ldx, K, n_rows, n_rows_dev, rowptr, col, reduce, wl, wr, bias, Fo,
                             out, ldo, relu, p_drop, seed, seed_dev, nullptr, K, st, &rc, ldw,
                             nullptr, 0, x_dev, exact, z, ldz, xrow, xrow_dev, x_rows, col_x, x_bf16,
                             w_bf16, false, false, false, n_edge_rows, n_edge_rows_dev, img_ws)) {
            if (rc) return rc;
            return narrow_agg_launch(z, ldz, Fo, rowptr, col, n_rows, n_rows_dev, n_edge_rows,
                                     n_edge_rows_dev, reduce, out, ldo, st, nullptr);
        }
    }
    // wide layers (the row-tile kernel's weight image too large for its LDS,
    // or K % 4 != 0): aggregate launch + 2-D tiled dual GEMM
    // (x_dev: a graph slot's batch rows in place -- K % 4 != 0 rows too, the
    // wide kernels load them at 4-B alignment)
    if ((x || x_dev) && !xrow && !xrow_dev && !x_bf16 && !out_bf16 && sage_wide_preferred(K, Fo, exact) &&
        (agg_out || !wl || ws_bytes >= sage_wide_workspace_bytes(K, n_edge_rows)))
        return sage_fwd_wide(x, ldx, K, n_rows, n_rows_dev, n_edge_rows, n_edge_rows_dev, rowptr,
                             col, reduce, wl, wr, ldw, bias, Fo, out, ldo, relu, p_drop, seed,
                             seed_dev, agg_out, ld_agg, ws, ws_bytes, st, exact, x_dev);
    // max layers with a wide input: the aggregate by its own launch (a wave per
    // row, every column in flight) into the saved-aggregate buffer, which the
    // row-tile kernel's edge tiles then read densely -- its in-kernel gather
    // walks 16-row tiles one 128-column chunk at a time (Amazon-Computers'
    // 512 -> 10 layer: 67 us for ~3k rows with in-edges)
    // NGNN_AGGPRE (read once; A/B): 1 -- mean / sum layers too (layer 0 of
    // products: its 16.2 k rows with in-edges gathered at full occupancy
    // instead of inside the row-tile kernel, one wave per 16-row tile)
    static const int aggpre_all = [] {
        const char *e = std::getenv("NGNN_AGGPRE");
        return e ? std::atoi(e) : 0;
    }();
    const bool agg_pre = (reduce == NGNN_REDUCE_MAX ? K >= 256 : aggpre_all == 1) && wl && agg_out &&
                         (x || x_dev) && !xrow && !xrow_dev && !x_bf16 && ld_agg % 4 == 0 &&
                         aligned(agg_out, 16);
    if (agg_pre) {
        rc = sage_wide_aggregate(x, ldx, K, n_rows, n_rows_dev, n_edge_rows, n_edge_rows_dev, rowptr,
                                 col, reduce, agg_out, ld_agg, st, x_dev);
        if (rc) return rc;
    }
    if (!sage_fwd_rowtile(x, ldx, K, n_rows, n_rows_dev, rowptr, col, reduce, wl, wr, bias, Fo, out,
                          ldo, relu, p_drop, seed, seed_dev, agg_out, ld_agg, st, &rc, ldw, ws,
                          ws_bytes, x_dev, exact, nullptr, 0, xrow, xrow_dev, x_rows, col_x, x_bf16,
                          w_bf16, wl_prepacked, agg_pre, out_bf16, n_edge_rows, n_edge_rows_dev,
                          img_ws))
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
