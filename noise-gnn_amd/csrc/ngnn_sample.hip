// One hop of uniform neighbour sampling without replacement on the device.
//
// Stands in for the sampler PyG's NeighborLoader runs in a worker process
// (pyg-lib / torch-sparse neighbor_sample [ext], constructed at
// pipeline.py:75-83, pipeline_s.py:72-80): for every frontier node take
// min(deg, fanout) distinct in-neighbours uniformly at random; nodes with
// deg <= fanout keep all neighbours in CSR order.  The graph CSR stays
// resident in HBM (products: 123.7 M int32 columns ~ 495 MB), so no host
// sampling and no per-batch H2D copy of the block structure.
//
// Floyd's algorithm: k draws, each O(k) duplicate check in registers
// (fanout <= 64); one thread per frontier node, counter-based RNG keyed by
// (seed, frontier position, draw) so results do not depend on scheduling.
#include <algorithm>

#include "ngnn_internal.h"

namespace ngnn {
namespace {

constexpr int kMaxFanout = 64;
constexpr int kMaxHops = 8;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// min(d, k) distinct CSR positions of a degree-d row, Floyd order; d <= k:
// all positions in CSR order.  Keyed by (seed, frontier position i).
__device__ __forceinline__ int floyd_sample(int64_t d, int fanout, uint64_t seed, int64_t i,
                                            int64_t (&sel)[kMaxFanout]) {
    const int k = d < fanout ? static_cast<int>(d) : fanout;
    if (d <= fanout) {
        for (int j = 0; j < k; ++j) sel[j] = j;
        return k;
    }
    const uint64_t base = mix64(seed ^ mix64(static_cast<uint64_t>(i) + 0x632BE59BD9B4E019ull));
    int m = 0;
    for (int64_t j = d - k; j < d; ++j) {
        const uint64_t r = mix64(base + static_cast<uint64_t>(j));
        const int64_t t = static_cast<int64_t>(
            (static_cast<unsigned __int128>(r) * static_cast<uint64_t>(j + 1)) >> 64);
        bool dup = false;
        for (int q = 0; q < m; ++q) dup |= sel[q] == t;
        sel[m++] = dup ? j : t;
    }
    return k;
}

__global__ __launch_bounds__(256) void k_sample_hop(const int64_t *__restrict__ rowptr,
                                                    const int32_t *__restrict__ gcol,
                                                    const int64_t *__restrict__ frontier,
                                                    int64_t nf, int fanout, uint64_t seed,
                                                    int64_t *__restrict__ out_nbr,
                                                    int32_t *__restrict__ out_cnt) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= nf) return;
    const int64_t v = frontier[i];
    const int64_t b = rowptr[v];
    int64_t sel[kMaxFanout];
    const int k = floyd_sample(rowptr[v + 1] - b, fanout, seed, i, sel);
    int64_t *o = out_nbr + i * fanout;
    for (int q = 0; q < k; ++q) o[q] = gcol[b + sel[q]];
    for (int j = k; j < fanout; ++j) o[j] = -1;
    out_cnt[i] = k;
}

// ---------------------------------------------------------------------------
// Whole-block sampler (ngnn_sample_block): every hop, the relabelling to
// local ids and the block's edge list on the device, no host round trip
// until the final counts.  Local ids follow NeighborLoader's contract: seeds
// first, then each hop's newly reached nodes in order of FIRST appearance in
// the hop's (frontier position, draw) sequence.
//
// Persistent map (caller-owned, int32 [2 * n_graph], all -1 between calls):
//   map[v]            local id of global node v in the current block, or -1
//   map[n_graph + v]  claim: INT32_MAX - (first hop position at which v
//                     appeared while unmapped), by atomicMax; -1 = none
// The finish call restores every entry it touched to -1.
//
// Per-hop state (int32 x4 in the workspace): {lo, hi, e0, -}: the hop's
// frontier is local ids [lo, hi), its edges start at e0.

constexpr int kSbBlock = 256;

struct SbWs {  // carved from the caller's workspace
    int32_t *state;  // [4 * (H + 1)]
    int32_t *cand;   // [sum_h nf_cap_h * f_h]  global ids of each hop's draws
    int32_t *cnt;    // [sum_h nf_cap_h]
    uint64_t *lb;    // [max_h nblk_h + 1]     per-tile look-back words + the tile ticket
    int32_t *nid;    // [n_cap]                local -> global
    int32_t *esrc;   // [e_cap]
    int32_t *edst;   // [e_cap]
};

__global__ __launch_bounds__(kSbBlock) void k_sb_init(const int64_t *__restrict__ seeds, int B,
                                                      int32_t *__restrict__ map,
                                                      int32_t *__restrict__ nid,
                                                      int32_t *__restrict__ state) {
    const int i = blockIdx.x * kSbBlock + threadIdx.x;
    if (i < B) {
        const int32_t v = static_cast<int32_t>(seeds[i]);
        map[v] = i;
        nid[i] = v;
    }
    if (i == 0) {
        state[0] = 0;
        state[1] = B;
        state[2] = 0;
        state[3] = 0;
    }
}

// Floyd draws with the fanout bounded at compile time (KF >= fanout): the
// selections stay in registers (fully unrolled), so a node's column and map
// loads issue back to back instead of as one dependent chain through
// scratch.  Same draws as floyd_sample.
template <int KF>
__device__ __forceinline__ int floyd_sample_r(int64_t d, int fanout, uint64_t seed, int64_t i,
                                              int32_t (&sel)[KF]) {
    const int k = d < fanout ? static_cast<int>(d) : fanout;
    if (d <= fanout) {
#pragma unroll
        for (int j = 0; j < KF; ++j) sel[j] = j;
        return k;
    }
    const uint64_t base = mix64(seed ^ mix64(static_cast<uint64_t>(i) + 0x632BE59BD9B4E019ull));
#pragma unroll
    for (int jj = 0; jj < KF; ++jj) {
        if (jj < k) {
            const int64_t j = d - k + jj;
            const uint64_t r = mix64(base + static_cast<uint64_t>(j));
            const int64_t t = static_cast<int64_t>(
                (static_cast<unsigned __int128>(r) * static_cast<uint64_t>(j + 1)) >> 64);
            bool dup = false;
#pragma unroll
            for (int q = 0; q < jj; ++q) dup |= sel[q] == t;
            sel[jj] = static_cast<int32_t>(dup ? j : t);
        }
    }
    return k;
}

// draws of frontier node i -> cand[i*f + j]; claims first appearances.
// Also (round 6, one launch fewer per hop): the previous hop's edges
// relabelled to local ids (its assignment is complete: the launch before),
// and this hop's look-back words and tile ticket cleared for k_sb_assign_lb.
template <int KF>
__global__ __launch_bounds__(kSbBlock) void k_sb_sample(
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ gcol, int64_t n_graph,
    const int32_t *__restrict__ hs, const int32_t *__restrict__ nid, int fanout, uint64_t seed,
    int32_t *__restrict__ cand, int32_t *__restrict__ cnt, int32_t *__restrict__ map,
    const int32_t *__restrict__ hs_prev, int32_t *__restrict__ esrc, uint64_t *__restrict__ lb, int nblk) {
    const int i = blockIdx.x * kSbBlock + threadIdx.x;
    const int stride = gridDim.x * kSbBlock;
    for (int t = i; t <= nblk; t += stride) lb[t] = 0;  // (lb[nblk]: the tile ticket)
    if (hs_prev)  // edges of the previous hop [hs_prev[2], hs_prev[6])
        for (int e = hs_prev[2] + i; e < hs_prev[6]; e += stride) esrc[e] = map[esrc[e]];
    const int lo = hs[0], hi = hs[1];
    if (i >= hi - lo) return;
    const int64_t v = nid[lo + i];
    const int64_t b = rowptr[v];
    int32_t sel[KF];
    const int k = floyd_sample_r<KF>(rowptr[v + 1] - b, fanout, seed, i, sel);
    int32_t u[KF], mp[KF];
#pragma unroll
    for (int j = 0; j < KF; ++j)
        if (j < k) u[j] = gcol[b + sel[j]];
#pragma unroll
    for (int j = 0; j < KF; ++j)
        if (j < k) {
            cand[i * fanout + j] = u[j];
            mp[j] = map[u[j]];
        }
    int32_t *claim = map + n_graph;
#pragma unroll
    for (int j = 0; j < KF; ++j)
        if (j < k && mp[j] < 0) atomicMax(claim + u[j], INT32_MAX - (i * fanout + j));
    cnt[i] = k;
}

// first-appearance flags of frontier node i's draws (bit j), and the draws
template <int KF>
__device__ __forceinline__ uint64_t sb_new_flags(const int32_t *cand, const int32_t *map,
                                                 const int32_t *claim, int i, int fanout, int k,
                                                 int32_t (&u)[KF]) {
    int32_t c[KF], m[KF];
#pragma unroll
    for (int j = 0; j < KF; ++j)
        if (j < k) u[j] = cand[i * fanout + j];
#pragma unroll
    for (int j = 0; j < KF; ++j)
        if (j < k) {
            c[j] = claim[u[j]];
            m[j] = map[u[j]];
        }
    uint64_t f = 0;
#pragma unroll
    for (int j = 0; j < KF; ++j)
        if (j < k && c[j] == INT32_MAX - (i * fanout + j) && m[j] < 0) f |= 1ull << j;
    return f;
}

__device__ __forceinline__ int block_excl_scan(int v, int *sh) {
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int o = 1; o < kSbBlock; o <<= 1) {
        const int a = t >= o ? sh[t - o] : 0;
        __syncthreads();
        sh[t] += a;
        __syncthreads();
    }
    const int r = sh[t] - v;
    __syncthreads();
    return r;
}

// look-back word of a tile: status (bits 62-63: 1 aggregate, 2 inclusive
// prefix) | new nodes (bits 31-61) | edges (bits 0-30); counts < 2^30
// (sb_plan bounds n, e by INT32_MAX / 2)
constexpr uint64_t kLbAgg = 1ull << 62, kLbPre = 2ull << 62;
__device__ __forceinline__ uint64_t lb_word(uint64_t st, int e, int n) {
    return st | (static_cast<uint64_t>(n) << 31) | static_cast<uint64_t>(e);
}

// One hop's relabelling in ONE launch (round 6; was count + scan + assign):
// each tile (256 frontier positions, in ticket order -- a tile only waits
// for tiles that already run) takes its positions' draws and first-
// appearance flags, publishes its (edges, new nodes) counts, finds its
// exclusive prefix by a decoupled look-back over the tiles before it, then
// assigns the new local ids (map, nid) in (position, draw) order and writes
// the hop's edges (global sources, local targets).  The last tile writes the
// next hop's state.  Same ids and edge order as the three launches.
template <int KF>
__global__ __launch_bounds__(kSbBlock) void k_sb_assign_lb(
    int32_t *__restrict__ hs, const int32_t *__restrict__ cand, const int32_t *__restrict__ cnt,
    int32_t *__restrict__ map, int64_t n_graph, int fanout, uint64_t *__restrict__ lb, int nblk,
    int32_t *__restrict__ nid, int32_t *__restrict__ esrc, int32_t *__restrict__ edst) {
    __shared__ int sh[kSbBlock];
    __shared__ int s_tile, s_pe, s_pn;
    if (threadIdx.x == 0)
        s_tile = static_cast<int>(atomicAdd(reinterpret_cast<unsigned long long *>(lb + nblk), 1ull));
    __syncthreads();
    const int tile = s_tile;
    const int i = tile * kSbBlock + threadIdx.x;
    const int lo = hs[0], hi = hs[1], e0 = hs[2];
    const int nf = hi - lo;
    int k = 0;
    uint64_t fl = 0;
    int32_t u[KF];
    if (i < nf) {
        k = cnt[i];
        // race-free although other tiles write map[] meanwhile: only the
        // position that won u's claim ever writes map[u] (after reading
        // it), and for every other position the flag is false whatever
        // map[u] reads
        fl = sb_new_flags<KF>(cand, map, map + n_graph, i, fanout, k, u);
    }
    const int xe = block_excl_scan(k, sh);
    const int nn = __popcll(fl);
    const int xn = block_excl_scan(nn, sh);
    // tile totals: the last thread's exclusive value plus its own
    __shared__ int s_te, s_tn;
    if (threadIdx.x == kSbBlock - 1) {
        s_te = xe + k;
        s_tn = xn + nn;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int ae = s_te, an = s_tn;
        int pe = 0, pn = 0;
        if (tile == 0) {
            __hip_atomic_store(lb + tile, lb_word(kLbPre, ae, an), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(lb + tile, lb_word(kLbAgg, ae, an), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            for (int p = tile - 1; p >= 0;) {
                const uint64_t w = __hip_atomic_load(lb + p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                const uint64_t st = w & (3ull << 62);
                if (st == 0) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                pe += static_cast<int>(w & 0x7FFFFFFFull);
                pn += static_cast<int>((w >> 31) & 0x7FFFFFFFull);
                if (st == kLbPre) break;
                --p;
            }
            __hip_atomic_store(lb + tile, lb_word(kLbPre, pe + ae, pn + an), __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        s_pe = pe;
        s_pn = pn;
        if (tile == nblk - 1) {  // the next hop's state: this hop's new nodes, its edges' end
            hs[4] = hi;
            hs[5] = hi + pn + an;
            hs[6] = e0 + pe + ae;
            hs[7] = 0;
        }
    }
    __syncthreads();
    int e = e0 + s_pe + xe;
    int n = hi + s_pn + xn;
#pragma unroll
    for (int j = 0; j < KF; ++j) {
        if (j < k) {
            if ((fl >> j) & 1) {
                map[u[j]] = n;
                nid[n++] = u[j];
            }
            esrc[e + j] = u[j];
            edst[e + j] = lo + i;
        }
    }
}

// the last hop's edges relabelled; counts = {n_total, e_total, n_active, -}
__global__ __launch_bounds__(kSbBlock) void k_sb_tail(const int32_t *__restrict__ state, int H,
                                                      const int32_t *__restrict__ map,
                                                      int32_t *__restrict__ esrc, int32_t *__restrict__ counts) {
    const int i = blockIdx.x * kSbBlock + threadIdx.x;
    if (H > 0) {
        const int32_t *hl = state + 4 * (H - 1);
        for (int e = hl[2] + i; e < hl[6]; e += gridDim.x * kSbBlock) esrc[e] = map[esrc[e]];
    }
    if (i == 0) {
        counts[0] = state[4 * H + 1];
        counts[1] = state[4 * H + 2];
        counts[2] = state[4 * (H > 0 ? H - 1 : 0) + 1];
        counts[3] = 0;
    }
}

// outputs + map reset: n_id (int64), y = y_all[n_id], edge_index [2, E]
__global__ __launch_bounds__(kSbBlock) void k_sb_finish(
    const int32_t *__restrict__ nid, int n, const int32_t *__restrict__ esrc,
    const int32_t *__restrict__ edst, int E, int32_t *__restrict__ map, int64_t n_graph,
    int64_t *__restrict__ n_id, const int64_t *__restrict__ y_all, int64_t *__restrict__ y,
    int64_t *__restrict__ ei) {
    const int64_t stride = (int64_t)gridDim.x * kSbBlock;
    for (int64_t t = blockIdx.x * (int64_t)kSbBlock + threadIdx.x; t < max(n, E); t += stride) {
        if (t < n) {
            const int32_t u = nid[t];
            n_id[t] = u;
            if (y) y[t] = y_all[u];
            map[u] = -1;
            map[n_graph + u] = -1;
        }
        if (t < E) {
            ei[t] = esrc[t];
            ei[E + t] = edst[t];
        }
    }
}

// x[i] = x_all[n_id[i]], 16-B vectors (F % 4 == 0, aligned rows); 32-bit
// item indices (n * F/4 < 2^31 checked by the caller), one vector per thread
__global__ __launch_bounds__(kSbBlock) void k_gather_rows4(const float *__restrict__ x_all,
                                                           int64_t ldx, const int32_t *__restrict__ nid,
                                                           int n, int f4, float *__restrict__ x,
                                                           int64_t ldo) {
    const int total = n * f4;
    for (int t = blockIdx.x * kSbBlock + threadIdx.x; t < total; t += gridDim.x * kSbBlock) {
        const int r = t / f4, c = (t - r * f4) * 4;
        *reinterpret_cast<float4 *>(x + static_cast<int64_t>(r) * ldo + c) =
            *reinterpret_cast<const float4 *>(x_all + static_cast<int64_t>(nid[r]) * ldx + c);
    }
}

// the block's outputs in ONE launch (round 6): blocks [0, gx) gather x rows
// (k_gather_rows4's work), the rest k_sb_finish's (ids, labels, edges, map
// reset -- the gather reads nid only, so the two roles need no order)
__global__ __launch_bounds__(kSbBlock) void k_sb_out(const float *__restrict__ x_all, int64_t ldx,
                                                     const int32_t *__restrict__ nid, int n, int f4,
                                                     float *__restrict__ x, int64_t ldo, int gx,
                                                     const int32_t *__restrict__ esrc, const int32_t *__restrict__ edst,
                                                     int E, int32_t *__restrict__ map, int64_t n_graph,
                                                     int64_t *__restrict__ n_id, const int64_t *__restrict__ y_all,
                                                     int64_t *__restrict__ y, int64_t *__restrict__ ei) {
    if (static_cast<int>(blockIdx.x) < gx) {
        const int total = n * f4;
        for (int t = blockIdx.x * kSbBlock + threadIdx.x; t < total; t += gx * kSbBlock) {
            const int r = t / f4, c = (t - r * f4) * 4;
            *reinterpret_cast<float4 *>(x + static_cast<int64_t>(r) * ldo + c) =
                *reinterpret_cast<const float4 *>(x_all + static_cast<int64_t>(nid[r]) * ldx + c);
        }
        return;
    }
    const int64_t stride = static_cast<int64_t>(gridDim.x - gx) * kSbBlock;
    for (int64_t t = (blockIdx.x - gx) * static_cast<int64_t>(kSbBlock) + threadIdx.x; t < max(n, E); t += stride) {
        if (t < n) {
            const int32_t u = nid[t];
            n_id[t] = u;
            if (y) y[t] = y_all[u];
            map[u] = -1;
            map[n_graph + u] = -1;
        }
        if (t < E) {
            ei[t] = esrc[t];
            ei[E + t] = edst[t];
        }
    }
}

__global__ __launch_bounds__(kSbBlock) void k_gather_rows1(const float *__restrict__ x_all,
                                                           int64_t ldx, const int32_t *__restrict__ nid,
                                                           int64_t n, int64_t F,
                                                           float *__restrict__ x, int64_t ldo) {
    const int64_t stride = (int64_t)gridDim.x * kSbBlock;
    for (int64_t t = blockIdx.x * (int64_t)kSbBlock + threadIdx.x; t < n * F; t += stride) {
        const int64_t r = t / F, c = t - r * F;
        x[r * ldo + c] = x_all[nid[r] * ldx + c];
    }
}

struct SbPlan {
    int64_t n_cap, e_cap, nf_cap[kMaxHops], cand_off[kMaxHops], cnt_off[kMaxHops], max_nblk;
    size_t bytes;
    size_t off_state, off_cand, off_cnt, off_bsum, off_nid, off_esrc, off_edst;
};

// capacities: frontier_h <= B prod_{j<h} f_j, all within int32
bool sb_plan(int64_t B, const int32_t *fanouts, int H, SbPlan *p) {
    if (B < 0 || H < 0 || H > kMaxHops) return false;
    int64_t nf = B, n = B, e = 0, cand = 0, cntn = 0, nblk = 1;
    for (int h = 0; h < H; ++h) {
        const int64_t f = fanouts[h];
        if (f < 0 || f > kMaxFanout) return false;
        p->nf_cap[h] = nf;
        p->cand_off[h] = cand;
        p->cnt_off[h] = cntn;
        cand += nf * f;
        cntn += nf;
        nblk = std::max<int64_t>(nblk, ceil_div(nf, kSbBlock));
        e += nf * f;
        nf *= f;
        n += nf;
        if (n > INT32_MAX / 2 || e > INT32_MAX / 2) return false;
    }
    p->n_cap = n;
    p->e_cap = e;
    p->max_nblk = nblk;
    size_t o = 0;
    auto take = [&](size_t words) {
        const size_t r = o;
        o += ((words * 4 + 255) / 256) * 256;
        return r;
    };
    p->off_state = take(4 * (H + 1));
    p->off_cand = take(static_cast<size_t>(std::max<int64_t>(cand, 1)));
    p->off_cnt = take(static_cast<size_t>(std::max<int64_t>(cntn, 1)));
    p->off_bsum = take(static_cast<size_t>(2 * (nblk + 1)));
    p->off_nid = take(static_cast<size_t>(n));
    p->off_esrc = take(static_cast<size_t>(std::max<int64_t>(e, 1)));
    p->off_edst = take(static_cast<size_t>(std::max<int64_t>(e, 1)));
    p->bytes = o;
    return true;
}

SbWs sb_carve(void *ws, const SbPlan &p) {
    char *b = static_cast<char *>(ws);
    return SbWs{reinterpret_cast<int32_t *>(b + p.off_state), reinterpret_cast<int32_t *>(b + p.off_cand),
                reinterpret_cast<int32_t *>(b + p.off_cnt), reinterpret_cast<uint64_t *>(b + p.off_bsum),
                reinterpret_cast<int32_t *>(b + p.off_nid), reinterpret_cast<int32_t *>(b + p.off_esrc),
                reinterpret_cast<int32_t *>(b + p.off_edst)};
}

}  // namespace
}  // namespace ngnn

using namespace ngnn;

extern "C" int ngnn_sample_hop(const int64_t *g_rowptr, const int32_t *g_col,
                               const int64_t *frontier, int64_t n_frontier, int fanout,
                               uint64_t seed, int64_t *out_nbr, int32_t *out_cnt, void *stream) {
    NGNN_RETURN_IF(n_frontier < 0 || fanout < 0, NGNN_E_ARG);
    NGNN_RETURN_IF(fanout > kMaxFanout, NGNN_E_SHAPE);
    if (n_frontier == 0 || fanout == 0) return NGNN_OK;
    NGNN_RETURN_IF(!g_rowptr || !g_col || !frontier || !out_nbr || !out_cnt, NGNN_E_ARG);
    hipLaunchKernelGGL(k_sample_hop, dim3(ceil_div(n_frontier, 256)), dim3(256), 0,
                       as_stream(stream), g_rowptr, g_col, frontier, n_frontier, fanout, seed,
                       out_nbr, out_cnt);
    return launch_status();
}

extern "C" size_t ngnn_sample_block_workspace_bytes(int64_t batch, const int32_t *fanouts,
                                                    int n_hops) {
    SbPlan p;
    if (!fanouts && n_hops > 0) return 0;
    return sb_plan(batch, fanouts, n_hops, &p) ? p.bytes : 0;
}

extern "C" int ngnn_sample_block(const int64_t *g_rowptr, const int32_t *g_col, int64_t n_graph,
                                 const int64_t *seeds, int64_t n_seeds, const int32_t *fanouts,
                                 int n_hops, uint64_t seed, int32_t *node_map, void *ws,
                                 size_t ws_bytes, int32_t *counts, void *stream) {
    NGNN_RETURN_IF(n_graph < 0 || n_seeds < 0 || n_hops < 0 || (n_hops > 0 && !fanouts), NGNN_E_ARG);
    NGNN_RETURN_IF(!fits_i32(n_graph) || !fits_i32(n_seeds), NGNN_E_RANGE);
    SbPlan p;
    NGNN_RETURN_IF(!sb_plan(n_seeds, fanouts, n_hops, &p), NGNN_E_SHAPE);
    NGNN_RETURN_IF(!ws || ws_bytes < p.bytes, NGNN_E_WORKSPACE);
    NGNN_RETURN_IF(!node_map || !counts || (n_seeds > 0 && !seeds), NGNN_E_ARG);
    NGNN_RETURN_IF(n_hops > 0 && (!g_rowptr || !g_col), NGNN_E_ARG);
    hipStream_t st = as_stream(stream);
    const SbWs w = sb_carve(ws, p);
    hipLaunchKernelGGL(k_sb_init, dim3(std::max<int64_t>(1, ceil_div(n_seeds, kSbBlock))),
                       dim3(kSbBlock), 0, st, seeds, static_cast<int>(n_seeds), node_map, w.nid,
                       w.state);
    for (int h = 0; h < n_hops; ++h) {
        const int f = fanouts[h];
        const int kf = f <= 8 ? 8 : f <= 16 ? 16 : f <= 32 ? 32 : 64;
        int32_t *hs = w.state + 4 * h;
        const int64_t nf = p.nf_cap[h];
        const int nblk = static_cast<int>(std::max<int64_t>(1, ceil_div(nf, kSbBlock)));
        int32_t *cand = w.cand + p.cand_off[h], *cnt = w.cnt + p.cnt_off[h];
        // the per-hop seed of ngnn_sample_hop's callers (loader.sample_block)
        const uint64_t hseed = seed * 1000003ull + static_cast<uint64_t>(h);
        // two launches per hop (round 6; five before): draws + claims (+ the
        // previous hop's relabel), then the look-back relabelling
        auto hop = [&](auto kf_c) {
            constexpr int KF = decltype(kf_c)::value;
            hipLaunchKernelGGL(k_sb_sample<KF>, dim3(nblk), dim3(kSbBlock), 0, st, g_rowptr, g_col, n_graph, hs, w.nid,
                               f, hseed, cand, cnt, node_map, h > 0 ? hs - 4 : nullptr, w.esrc, w.lb, nblk);
            hipLaunchKernelGGL(k_sb_assign_lb<KF>, dim3(nblk), dim3(kSbBlock), 0, st, hs, cand, cnt, node_map,
                               n_graph, f, w.lb, nblk, w.nid, w.esrc, w.edst);
        };
        switch (kf) {
            case 8: hop(std::integral_constant<int, 8>{}); break;
            case 16: hop(std::integral_constant<int, 16>{}); break;
            case 32: hop(std::integral_constant<int, 32>{}); break;
            default: hop(std::integral_constant<int, 64>{}); break;
        }
    }
    // the last hop's relabel + counts = {n_total, e_total, n_active (rows that received edges), -}
    const int64_t e_last = n_hops > 0 ? p.nf_cap[n_hops - 1] * fanouts[n_hops - 1] : 0;
    hipLaunchKernelGGL(k_sb_tail, dim3(static_cast<unsigned>(std::clamp<int64_t>(ceil_div(e_last, kSbBlock), 1, 4096))),
                       dim3(kSbBlock), 0, st, w.state, n_hops, node_map, w.esrc, counts);
    return launch_status();
}

extern "C" int ngnn_sample_block_finish(const int32_t *fanouts, int n_hops, int64_t n_seeds,
                                        int64_t n_nodes, int64_t n_edges, int32_t *node_map,
                                        int64_t n_graph, const void *ws, size_t ws_bytes,
                                        int64_t *n_id, int64_t *edge_index, const int64_t *y_all,
                                        int64_t *y, const float *x_all, int64_t ldx, int64_t F,
                                        float *x, int64_t ldo, void *stream) {
    SbPlan p;
    NGNN_RETURN_IF(n_hops < 0 || (n_hops > 0 && !fanouts), NGNN_E_ARG);
    NGNN_RETURN_IF(!sb_plan(n_seeds, fanouts, n_hops, &p), NGNN_E_SHAPE);
    NGNN_RETURN_IF(!ws || ws_bytes < p.bytes, NGNN_E_WORKSPACE);
    NGNN_RETURN_IF(n_nodes < n_seeds || n_nodes > p.n_cap || n_edges < 0 || n_edges > p.e_cap,
                   NGNN_E_SHAPE);
    NGNN_RETURN_IF(!node_map || !n_id || (n_edges > 0 && !edge_index) || (y && !y_all), NGNN_E_ARG);
    NGNN_RETURN_IF(x && (!x_all || F <= 0 || ldx < F || ldo < F), NGNN_E_ARG);
    hipStream_t st = as_stream(stream);
    const SbWs w = sb_carve(const_cast<void *>(ws), p);
    const int64_t work = std::max<int64_t>(std::max<int64_t>(n_nodes, n_edges), 1);
    const unsigned gf = static_cast<unsigned>(std::min<int64_t>(ceil_div(work, kSbBlock), 4096));
    const bool vec = x && n_nodes > 0 && F % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0 && aligned(x_all, 16) &&
                     aligned(x, 16) && n_nodes * (F / 4) < INT32_MAX;
    if (vec) {  // the gather and the outputs in one launch
        const int gx = static_cast<int>(std::min<int64_t>(ceil_div(n_nodes * (F / 4), kSbBlock), 4096));
        hipLaunchKernelGGL(k_sb_out, dim3(gx + gf), dim3(kSbBlock), 0, st, x_all, ldx, w.nid,
                           static_cast<int>(n_nodes), static_cast<int>(F / 4), x, ldo, gx, w.esrc, w.edst,
                           static_cast<int>(n_edges), node_map, n_graph, n_id, y_all, y, edge_index);
        return launch_status();
    }
    if (x && n_nodes > 0) {  // gather before the map reset (order irrelevant: reads nid only)
        const int64_t items = vec ? n_nodes * (F / 4) : n_nodes * F;
        const unsigned grid = static_cast<unsigned>(std::min<int64_t>(ceil_div(items, kSbBlock), 65536));
        if (vec)
            hipLaunchKernelGGL(k_gather_rows4, dim3(grid), dim3(kSbBlock), 0, st,
                               x_all, ldx, w.nid, static_cast<int>(n_nodes),
                               static_cast<int>(F / 4), x, ldo);
        else
            hipLaunchKernelGGL(k_gather_rows1, dim3(grid), dim3(kSbBlock), 0, st, x_all, ldx, w.nid,
                               n_nodes, F, x, ldo);
    }
    hipLaunchKernelGGL(k_sb_finish, dim3(gf), dim3(kSbBlock), 0, st, w.nid, static_cast<int>(n_nodes), w.esrc, w.edst,
                       static_cast<int>(n_edges), node_map, n_graph, n_id, y_all, y, edge_index);
    return launch_status();
}
