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
    uint64_t *masks;  // [max_h ntile_h][16][2]  per wave chunk: (drawn, first appearance) lane masks
    int32_t *tcnt;    // [max_h ntile_h][2]      per tile: (edges, new nodes)
    int32_t *nid;    // [n_cap]                local -> global
    int32_t *esrc;   // [e_cap]
    int32_t *edst;   // [e_cap]
    int32_t *rp;     // [n_cap]    first edge of each frontier row (the block's CSR row pointers)
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

// Lane-per-draw layout (round 6): frontier position i owns a group of KF
// lanes (KF = fanout rounded up to 8/16/32/64, a power of two dividing the
// wave), lane j its draw j.  The per-thread layout before it ran one thread
// per position -- 60 workgroups for a products hop-2 frontier, each thread a
// serial chain of draws, loads and atomics -- latency-bound at ~30 us a
// launch.  Floyd's draws are independent but for the duplicate test: draw q's
// final choice is known once draws < q are, so the group resolves them in
// fanout - 1 shuffle rounds (lane q's choice broadcast, later lanes compare).
// Same selections as floyd_sample.
template <int KF>
__device__ __forceinline__ int floyd_lane(int64_t d, int fanout, uint64_t seed, int i, int j, int &k) {
    k = d < fanout ? static_cast<int>(d) : fanout;
    if (d <= fanout) return j;
    const uint64_t base = mix64(seed ^ mix64(static_cast<uint64_t>(i) + 0x632BE59BD9B4E019ull));
    const int64_t J = d - k + j;  // (lanes j >= k compute a value nobody reads)
    const uint64_t r = mix64(base + static_cast<uint64_t>(J));
    const int32_t t = static_cast<int32_t>((static_cast<unsigned __int128>(r) * static_cast<uint64_t>(J + 1)) >> 64);
    const int32_t jw = static_cast<int32_t>(J);
    bool dup = false;
    for (int q = 0; q < k - 1; ++q) {  // (k is uniform over the group; every source lane is active)
        const int32_t fq = __shfl(dup ? jw : t, q, KF);
        dup |= j > q && fq == t;
    }
    return dup ? jw : t;
}

constexpr int kSbTile = 1024;  // k_sb_count / k_sb_write's tile: kSbTile / KF frontier positions
constexpr int kSbChunks = kSbTile / 64;  // its wave chunks

__host__ __device__ constexpr int sb_kf(int f) { return f <= 8 ? 8 : f <= 16 ? 16 : f <= 32 ? 32 : 64; }

// draw j of frontier node i -> cand[i*f + j]; claims first appearances.
// Also (one launch fewer per hop): the previous hop's edges relabelled to
// local ids (its assignment is complete: the launch before).
template <int KF>
__global__ __launch_bounds__(kSbBlock) void k_sb_sample(
    const int64_t *__restrict__ rowptr, const int32_t *__restrict__ gcol, int64_t n_graph,
    const int32_t *__restrict__ hs, const int32_t *__restrict__ nid, int fanout, uint64_t seed,
    int32_t *__restrict__ cand, int32_t *__restrict__ cnt, int32_t *__restrict__ map,
    const int32_t *__restrict__ hs_prev, int32_t *__restrict__ esrc) {
    const int gt = blockIdx.x * kSbBlock + threadIdx.x;
    const int stride = gridDim.x * kSbBlock;
    if (hs_prev)  // edges of the previous hop [hs_prev[2], hs_prev[6])
        for (int e = hs_prev[2] + gt; e < hs_prev[6]; e += stride) esrc[e] = map[esrc[e]];
    const int lo = hs[0], hi = hs[1];
    const int i = gt / KF, j = gt % KF;
    if (i >= hi - lo) return;  // (whole groups)
    const int64_t v = nid[lo + i];
    const int64_t b = rowptr[v];
    int k;
    const int s = floyd_lane<KF>(rowptr[v + 1] - b, fanout, seed, i, j, k);
    if (j < k) {
        const int32_t u = gcol[b + s];
        cand[i * fanout + j] = u;
        const int32_t m = map[u], c = map[n_graph + u];
        const int32_t mine = INT32_MAX - (i * fanout + j);
        // (the claim only grows: a hub drawn by thousands of positions takes
        // an atomic only from those that still beat the standing claim)
        if (m < 0 && c < mine) atomicMax(map + n_graph + u, mine);
    }
    if (j == 0) cnt[i] = k;
}

__device__ __forceinline__ int wave_sum(int v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// One hop's relabelling in two launches with no waiting between workgroups
// (round 6; the single-pass decoupled look-back before it spun on its
// predecessors' words, ~17-34 us alone and ~60 us while the training step
// held the CUs).  A tile is kSbTile lanes = (position, draw) pairs in order.
// k_sb_count: each draw's first-appearance flag (its position won the claim
// and the node has no local id yet), per wave chunk the two lane masks, per
// tile the (edges, new nodes) totals.  The claims are final (the launch
// before), and nothing writes map[] here -- race-free by construction.
template <int KF>
__global__ __launch_bounds__(kSbTile) void k_sb_count(const int32_t *__restrict__ hs, const int32_t *__restrict__ cand,
                                                      const int32_t *__restrict__ cnt, const int32_t *__restrict__ map,
                                                      int64_t n_graph, int fanout, uint64_t *__restrict__ masks,
                                                      int32_t *__restrict__ tcnt) {
    __shared__ int s_e[kSbChunks], s_n[kSbChunks];
    const int tile = blockIdx.x;
    const int gt = tile * kSbTile + threadIdx.x;
    const int i = gt / KF, j = gt % KF;
    const int nf = hs[1] - hs[0];
    bool has = false, fresh = false;
    if (i < nf && j < cnt[i]) {
        has = true;
        const int32_t u = cand[i * fanout + j];
        const int32_t c = map[n_graph + u], m = map[u];
        fresh = c == INT32_MAX - (i * fanout + j) && m < 0;
    }
    const uint64_t be = __ballot(has), bn = __ballot(fresh);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) {
        masks[2 * (tile * kSbChunks + wv)] = be;
        masks[2 * (tile * kSbChunks + wv) + 1] = bn;
        s_e[wv] = __popcll(be);
        s_n[wv] = __popcll(bn);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int e = 0, n = 0;
#pragma unroll
        for (int w = 0; w < kSbChunks; ++w) {
            e += s_e[w];
            n += s_n[w];
        }
        tcnt[2 * tile] = e;
        tcnt[2 * tile + 1] = n;
    }
}

// k_sb_write: the tile's exclusive prefix -- the totals of the tiles before
// it, summed by one wave -- and its chunks' prefixes (one wave scans the
// sixteen), then the new local ids (map, nid) in (position, draw) order, the
// hop's edges (global sources, local targets) and row pointers.  The last
// tile writes the next hop's state.
template <int KF>
__global__ __launch_bounds__(kSbTile) void k_sb_write(int32_t *__restrict__ hs, const int32_t *__restrict__ cand,
                                                      int32_t *__restrict__ map, int fanout,
                                                      const uint64_t *__restrict__ masks,
                                                      const int32_t *__restrict__ tcnt, int ntile,
                                                      int32_t *__restrict__ nid, int32_t *__restrict__ esrc,
                                                      int32_t *__restrict__ edst, int32_t *__restrict__ rp) {
    __shared__ int s_pe, s_pn;
    __shared__ int s_ce[kSbChunks], s_cn[kSbChunks];
    const int tile = blockIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int lo = hs[0], hi = hs[1], e0 = hs[2];
    const int nf = hi - lo;
    if (wv == 0) {
        int pe = 0, pn = 0;
        for (int b = lane; b < tile; b += 64) {
            pe += tcnt[2 * b];
            pn += tcnt[2 * b + 1];
        }
        pe = wave_sum(pe);
        pn = wave_sum(pn);
        if (lane == 0) {
            s_pe = pe;
            s_pn = pn;
            if (tile == ntile - 1) {  // the next hop's state: this hop's new nodes, its edges' end
                hs[4] = hi;
                hs[5] = hi + pn + tcnt[2 * tile + 1];
                hs[6] = e0 + pe + tcnt[2 * tile];
                hs[7] = 0;
            }
        }
    } else if (wv == 1) {
        const int c = tile * kSbChunks + (lane & (kSbChunks - 1));
        const int ce = lane < kSbChunks ? __popcll(masks[2 * c]) : 0;
        const int cn = lane < kSbChunks ? __popcll(masks[2 * c + 1]) : 0;
        int ie = ce, in = cn;
#pragma unroll
        for (int o = 1; o < kSbChunks; o <<= 1) {
            const int ae = __shfl_up(ie, o), an = __shfl_up(in, o);
            if (lane >= o) {
                ie += ae;
                in += an;
            }
        }
        if (lane < kSbChunks) {
            s_ce[lane] = ie - ce;
            s_cn[lane] = in - cn;
        }
    }
    __syncthreads();
    const int gt = tile * kSbTile + threadIdx.x;
    const int i = gt / KF, j = gt % KF;
    const uint64_t mh = masks[2 * (tile * kSbChunks + wv)], mf = masks[2 * (tile * kSbChunks + wv) + 1];
    const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
    const int e = e0 + s_pe + s_ce[wv] + __popcll(mh & below);
    if ((mh >> lane) & 1) {
        const int32_t u = cand[i * fanout + j];
        esrc[e] = u;
        edst[e] = lo + i;
        if ((mf >> lane) & 1) {
            const int n = hi + s_pn + s_cn[wv] + __popcll(mf & below);
            map[u] = n;
            nid[n] = u;
        }
    }
    if (j == 0 && i < nf) rp[lo + i] = e;  // (frontier row lo + i's edges start here: CSR row pointer)
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
// the block's outputs, item t of a grid-stride loop: n_id, y, the node map
// reset, edge_index; with csr_rp / csr_col (ABI 18, nullable): its
// target-grouped CSR (row pointers from the relabelling -- rows past the last
// frontier have no edges -- and the relabelled sources as int32), so a
// consumer builds none
// cnt (ABI 19, nullable): the block's {n, E, n_active} read on the device
// (the sampler's counts; n / E / n_act then hold the capacities the grid and
// the outputs are sized for, and bound the device values); ld_ei: edge_index's
// row stride
struct SbOut {
    const int32_t *nid, *esrc, *edst, *rp;
    int n, E, n_act;
    int32_t *map;
    int64_t n_graph;
    int64_t *n_id;
    const int64_t *y_all;
    int64_t *y, *ei;
    int32_t *csr_rp, *csr_col;
    int64_t ld_ei;
    const int32_t *cnt;
};
__device__ __forceinline__ void sb_counts(SbOut &o) {
    if (o.cnt) {
        o.n = min(o.cnt[0], o.n);
        o.E = min(o.cnt[1], o.E);
        o.n_act = min(o.cnt[2], o.n);
    }
}
__device__ __forceinline__ void sb_emit(const SbOut &o, int64_t t) {
    if (t < o.n) {
        const int32_t u = o.nid[t];
        o.n_id[t] = u;
        if (o.y) o.y[t] = o.y_all[u];
        o.map[u] = -1;
        o.map[o.n_graph + u] = -1;
    }
    if (t < o.E) {
        o.ei[t] = o.esrc[t];
        o.ei[o.ld_ei + t] = o.edst[t];
        if (o.csr_col) o.csr_col[t] = o.esrc[t];
    }
    // (no edges: every row pointer is 0 -- with no hops rp was never written)
    if (o.csr_rp && t <= o.n) o.csr_rp[t] = (t < o.n_act && o.E > 0) ? o.rp[t] : o.E;
}

__global__ __launch_bounds__(kSbBlock) void k_sb_finish(SbOut o) {
    sb_counts(o);
    const int64_t stride = (int64_t)gridDim.x * kSbBlock;
    for (int64_t t = blockIdx.x * (int64_t)kSbBlock + threadIdx.x; t <= max(o.n, o.E); t += stride) sb_emit(o, t);
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
__global__ __launch_bounds__(kSbBlock) void k_sb_out(const float *__restrict__ x_all, int64_t ldx, int f4,
                                                     float *__restrict__ x, int64_t ldo, int gx, SbOut o) {
    sb_counts(o);
    if (static_cast<int>(blockIdx.x) < gx) {
        const int total = o.n * f4;
        for (int t = blockIdx.x * kSbBlock + threadIdx.x; t < total; t += gx * kSbBlock) {
            const int r = t / f4, c = (t - r * f4) * 4;
            *reinterpret_cast<float4 *>(x + static_cast<int64_t>(r) * ldo + c) =
                *reinterpret_cast<const float4 *>(x_all + static_cast<int64_t>(o.nid[r]) * ldx + c);
        }
        return;
    }
    const int64_t stride = static_cast<int64_t>(gridDim.x - gx) * kSbBlock;
    for (int64_t t = (blockIdx.x - gx) * static_cast<int64_t>(kSbBlock) + threadIdx.x; t <= max(o.n, o.E); t += stride)
        sb_emit(o, t);
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
    size_t off_state, off_cand, off_cnt, off_bsum, off_nid, off_esrc, off_edst, off_rp;
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
        if (nf * sb_kf(static_cast<int>(f)) > INT32_MAX / 2) return false;  // (lane indices)
        nblk = std::max<int64_t>(nblk, ceil_div(nf * sb_kf(static_cast<int>(f)), kSbTile));
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
    p->off_bsum = take(static_cast<size_t>((2 * 2 * kSbChunks + 2) * nblk));  // masks + tile totals
    p->off_nid = take(static_cast<size_t>(n));
    p->off_esrc = take(static_cast<size_t>(std::max<int64_t>(e, 1)));
    p->off_edst = take(static_cast<size_t>(std::max<int64_t>(e, 1)));
    p->off_rp = take(static_cast<size_t>(n));
    p->bytes = o;
    return true;
}

SbWs sb_carve(void *ws, const SbPlan &p) {
    char *b = static_cast<char *>(ws);
    return SbWs{reinterpret_cast<int32_t *>(b + p.off_state), reinterpret_cast<int32_t *>(b + p.off_cand),
                reinterpret_cast<int32_t *>(b + p.off_cnt), reinterpret_cast<uint64_t *>(b + p.off_bsum),
                reinterpret_cast<int32_t *>(b + p.off_bsum + static_cast<size_t>(2 * kSbChunks * 8) * p.max_nblk),
                reinterpret_cast<int32_t *>(b + p.off_nid), reinterpret_cast<int32_t *>(b + p.off_esrc),
                reinterpret_cast<int32_t *>(b + p.off_edst), reinterpret_cast<int32_t *>(b + p.off_rp)};
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
        const int kf = sb_kf(f);
        int32_t *hs = w.state + 4 * h;
        const int64_t nf = p.nf_cap[h];
        // lane-per-draw grids: kf lanes per frontier position
        const int nblk = static_cast<int>(std::max<int64_t>(1, ceil_div(nf * kf, kSbTile)));
        const int sgrid = static_cast<int>(std::max<int64_t>(1, ceil_div(nf * kf, kSbBlock)));
        int32_t *cand = w.cand + p.cand_off[h], *cnt = w.cnt + p.cnt_off[h];
        // the per-hop seed of ngnn_sample_hop's callers (loader.sample_block)
        const uint64_t hseed = seed * 1000003ull + static_cast<uint64_t>(h);
        // three launches per hop (round 6; five before): draws + claims (+ the
        // previous hop's relabel), the first-appearance counts, the writes
        auto hop = [&](auto kf_c) {
            constexpr int KF = decltype(kf_c)::value;
            hipLaunchKernelGGL(k_sb_sample<KF>, dim3(sgrid), dim3(kSbBlock), 0, st, g_rowptr, g_col, n_graph, hs, w.nid,
                               f, hseed, cand, cnt, node_map, h > 0 ? hs - 4 : nullptr, w.esrc);
            hipLaunchKernelGGL(k_sb_count<KF>, dim3(nblk), dim3(kSbTile), 0, st, hs, cand, cnt, node_map, n_graph, f,
                               w.masks, w.tcnt);
            hipLaunchKernelGGL(k_sb_write<KF>, dim3(nblk), dim3(kSbTile), 0, st, hs, cand, node_map, f, w.masks,
                               w.tcnt, nblk, w.nid, w.esrc, w.edst, w.rp);
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
                                        float *x, int64_t ldo, int64_t n_active, int32_t *csr_rowptr,
                                        int32_t *csr_col, const int32_t *counts_dev, void *stream) {
    SbPlan p;
    NGNN_RETURN_IF(n_hops < 0 || (n_hops > 0 && !fanouts), NGNN_E_ARG);
    NGNN_RETURN_IF(!sb_plan(n_seeds, fanouts, n_hops, &p), NGNN_E_SHAPE);
    NGNN_RETURN_IF(!ws || ws_bytes < p.bytes, NGNN_E_WORKSPACE);
    NGNN_RETURN_IF(n_nodes < n_seeds || n_nodes > p.n_cap || n_edges < 0 || n_edges > p.e_cap,
                   NGNN_E_SHAPE);
    NGNN_RETURN_IF(!node_map || !n_id || (n_edges > 0 && !edge_index) || (y && !y_all), NGNN_E_ARG);
    NGNN_RETURN_IF(x && (!x_all || F <= 0 || ldx < F || ldo < F), NGNN_E_ARG);
    // (the CSR outputs come as a pair; a block without edges may pass no col)
    NGNN_RETURN_IF((!csr_rowptr && csr_col) || (csr_rowptr && !csr_col && n_edges > 0) || n_active < 0 ||
                       n_active > n_nodes,
                   NGNN_E_ARG);
    hipStream_t st = as_stream(stream);
    const SbWs w = sb_carve(const_cast<void *>(ws), p);
    const SbOut o{w.nid, w.esrc, w.edst, w.rp, static_cast<int>(n_nodes), static_cast<int>(n_edges),
                  static_cast<int>(n_active), node_map, n_graph, n_id, y_all, y, edge_index, csr_rowptr, csr_col,
                  n_edges, counts_dev};
    const int64_t work = std::max<int64_t>(std::max<int64_t>(n_nodes, n_edges), 1) + 1;
    const unsigned gf = static_cast<unsigned>(std::min<int64_t>(ceil_div(work, kSbBlock), 4096));
    const bool vec = x && n_nodes > 0 && F % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0 && aligned(x_all, 16) &&
                     aligned(x, 16) && n_nodes * (F / 4) < INT32_MAX;
    if (vec) {  // the gather and the outputs in one launch
        const int gx = static_cast<int>(std::min<int64_t>(ceil_div(n_nodes * (F / 4), kSbBlock), 4096));
        hipLaunchKernelGGL(k_sb_out, dim3(gx + gf), dim3(kSbBlock), 0, st, x_all, ldx, static_cast<int>(F / 4), x,
                           ldo, gx, o);
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
    hipLaunchKernelGGL(k_sb_finish, dim3(gf), dim3(kSbBlock), 0, st, o);
    return launch_status();
}
