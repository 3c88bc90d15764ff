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
    int32_t *bsum;   // [2 * max_h nblk_h]     per-block edge / new-node counts
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

// draws of frontier node i -> cand[i*f + j]; claims first appearances
template <int KF>
__global__ __launch_bounds__(kSbBlock) void k_sb_sample(
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ gcol, int64_t n_graph,
    const int32_t *__restrict__ hs, const int32_t *__restrict__ nid, int fanout, uint64_t seed,
    int32_t *__restrict__ cand, int32_t *__restrict__ cnt, int32_t *__restrict__ map) {
    const int i = blockIdx.x * kSbBlock + threadIdx.x;
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

__device__ __forceinline__ int block_sum(int v, int *red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    int t = 0;
    for (int j = 0; j < kSbBlock / 64; ++j) t += red[j];
    __syncthreads();
    return t;
}

template <int KF>
__global__ __launch_bounds__(kSbBlock) void k_sb_count(const int32_t *__restrict__ hs,
                                                       const int32_t *__restrict__ cand,
                                                       const int32_t *__restrict__ cnt,
                                                       const int32_t *__restrict__ map,
                                                       int64_t n_graph, int fanout,
                                                       int32_t *__restrict__ bsum, int nblk) {
    __shared__ int red[kSbBlock / 64];
    const int i = blockIdx.x * kSbBlock + threadIdx.x;
    const int nf = hs[1] - hs[0];
    int e = 0, n = 0;
    if (i < nf) {
        e = cnt[i];
        int32_t u[KF];
        n = __popcll(sb_new_flags<KF>(cand, map, map + n_graph, i, fanout, e, u));
    }
    e = block_sum(e, red);
    n = block_sum(n, red);
    if (threadIdx.x == 0) {
        bsum[blockIdx.x] = e;
        bsum[nblk + blockIdx.x] = n;
    }
}

// exclusive scan of the per-block counts (one workgroup) + next hop's state
__global__ __launch_bounds__(1024) void k_sb_scan(int32_t *__restrict__ hs, int32_t *__restrict__ bsum,
                                                  int nblk) {
    __shared__ int se[1024], sn[1024];
    const int t = threadIdx.x;
    const int per = (nblk + 1023) / 1024;
    const int b0 = min(nblk, t * per), b1 = min(nblk, b0 + per);
    int e = 0, n = 0;
    for (int b = b0; b < b1; ++b) {
        e += bsum[b];
        n += bsum[nblk + b];
    }
    se[t] = e;
    sn[t] = n;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
        const int ae = t >= o ? se[t - o] : 0, an = t >= o ? sn[t - o] : 0;
        __syncthreads();
        se[t] += ae;
        sn[t] += an;
        __syncthreads();
    }
    int pe = se[t] - e, pn = sn[t] - n;  // exclusive
    for (int b = b0; b < b1; ++b) {
        const int ve = bsum[b], vn = bsum[nblk + b];
        bsum[b] = pe;
        bsum[nblk + b] = pn;
        pe += ve;
        pn += vn;
    }
    if (t == 1023) {
        hs[4] = hs[1];           // next frontier: this hop's new nodes
        hs[5] = hs[1] + sn[t];
        hs[6] = hs[2] + se[t];
        hs[7] = 0;
    }
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

// new local ids (first appearances, in order) and the hop's edges
// (global source ids for now, local targets)
template <int KF>
__global__ __launch_bounds__(kSbBlock) void k_sb_assign(
    const int32_t *__restrict__ hs, const int32_t *__restrict__ cand, const int32_t *__restrict__ cnt,
    int32_t *__restrict__ map, int64_t n_graph, int fanout, const int32_t *__restrict__ bsum,
    int nblk, int32_t *__restrict__ nid, int32_t *__restrict__ esrc, int32_t *__restrict__ edst) {
    __shared__ int sh[kSbBlock];
    const int i = blockIdx.x * kSbBlock + threadIdx.x;
    const int lo = hs[0], hi = hs[1], e0 = hs[2];
    const int nf = hi - lo;
    int k = 0;
    uint64_t fl = 0;
    int32_t u[KF];
    if (i < nf) {
        k = cnt[i];
        // only the owner of u's claim ever writes map[u], and every flag is
        // read before this thread writes: the test is race-free
        fl = sb_new_flags<KF>(cand, map, map + n_graph, i, fanout, k, u);
    }
    int e = e0 + bsum[blockIdx.x] + block_excl_scan(k, sh);
    int n = hi + bsum[nblk + blockIdx.x] + block_excl_scan(__popcll(fl), sh);
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

__global__ __launch_bounds__(kSbBlock) void k_sb_relabel(const int32_t *__restrict__ hs,
                                                         const int32_t *__restrict__ map,
                                                         int32_t *__restrict__ esrc) {
    const int e = hs[2] + blockIdx.x * kSbBlock + threadIdx.x;
    if (e < hs[6]) esrc[e] = map[esrc[e]];
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

__global__ void k_sb_counts(const int32_t *__restrict__ state, int H, int32_t *__restrict__ counts) {
    if (threadIdx.x == 0) {
        counts[0] = state[4 * H + 1];
        counts[1] = state[4 * H + 2];
        counts[2] = state[4 * (H > 0 ? H - 1 : 0) + 1];
        counts[3] = 0;
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
    p->off_bsum = take(static_cast<size_t>(2 * nblk));
    p->off_nid = take(static_cast<size_t>(n));
    p->off_esrc = take(static_cast<size_t>(std::max<int64_t>(e, 1)));
    p->off_edst = take(static_cast<size_t>(std::max<int64_t>(e, 1)));
    p->bytes = o;
    return true;
}

SbWs sb_carve(void *ws, const SbPlan &p) {
    char *b = static_cast<char *>(ws);
    return SbWs{reinterpret_cast<int32_t *>(b + p.off_state), reinterpret_cast<int32_t *>(b + p.off_cand),
                reinterpret_cast<int32_t *>(b + p.off_cnt), reinterpret_cast<int32_t *>(b + p.off_bsum),
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
        if (f > 0) {
            auto sample = [&](auto kf_c) {
                constexpr int KF = decltype(kf_c)::value;
                hipLaunchKernelGGL(k_sb_sample<KF>, dim3(nblk), dim3(kSbBlock), 0, st, g_rowptr, g_col,
                                   n_graph, hs, w.nid, f, hseed, cand, cnt, node_map);
                hipLaunchKernelGGL(k_sb_count<KF>, dim3(nblk), dim3(kSbBlock), 0, st, hs, cand, cnt,
                                   node_map, n_graph, f, w.bsum, nblk);
            };
            switch (kf) {
                case 8: sample(std::integral_constant<int, 8>{}); break;
                case 16: sample(std::integral_constant<int, 16>{}); break;
                case 32: sample(std::integral_constant<int, 32>{}); break;
                default: sample(std::integral_constant<int, 64>{}); break;
            }
        } else {
            (void)hipMemsetAsync(w.bsum, 0, 2 * nblk * sizeof(int32_t), st);
        }
        hipLaunchKernelGGL(k_sb_scan, dim3(1), dim3(1024), 0, st, hs, w.bsum, nblk);
        if (f > 0) {
            auto assign = [&](auto kf_c) {
                constexpr int KF = decltype(kf_c)::value;
                hipLaunchKernelGGL(k_sb_assign<KF>, dim3(nblk), dim3(kSbBlock), 0, st, hs, cand, cnt,
                                   node_map, n_graph, f, w.bsum, nblk, w.nid, w.esrc, w.edst);
            };
            switch (kf) {
                case 8: assign(std::integral_constant<int, 8>{}); break;
                case 16: assign(std::integral_constant<int, 16>{}); break;
                case 32: assign(std::integral_constant<int, 32>{}); break;
                default: assign(std::integral_constant<int, 64>{}); break;
            }
            hipLaunchKernelGGL(k_sb_relabel, dim3(std::max<int64_t>(1, ceil_div(nf * f, kSbBlock))),
                               dim3(kSbBlock), 0, st, hs, node_map, w.esrc);
        }
    }
    // counts = {n_total, e_total, n_active (rows that received edges), -}
    hipLaunchKernelGGL(k_sb_counts, dim3(1), dim3(64), 0, st, w.state, n_hops, counts);
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
    if (x && n_nodes > 0) {  // gather before the map reset (order irrelevant: reads nid only)
        const bool vec = F % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0 && aligned(x_all, 16) &&
                         aligned(x, 16) && n_nodes * (F / 4) < INT32_MAX;
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
    hipLaunchKernelGGL(k_sb_finish,
                       dim3(static_cast<unsigned>(std::min<int64_t>(ceil_div(work, kSbBlock), 4096))),
                       dim3(kSbBlock), 0, st, w.nid, static_cast<int>(n_nodes), w.esrc, w.edst,
                       static_cast<int>(n_edges), node_map, n_graph, n_id, y_all, y, edge_index);
    return launch_status();
}
