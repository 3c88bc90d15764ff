// Static HIP-graph slot filling (ngnn/graphs.py): one launch copies a
// NeighborLoader block into the slot a captured training step reads.
//   rows  [0, N)        x copied (16-B vectors when rows allow), or with
//                       x_dev only its address stored (zero-copy)
//   edges [0, E)        copied;  [E, e_cap) padding self-loops on row
//                       N + floor(j (n_cap - N) / n_pad), j = e - E: targets
//                       stay non-decreasing (the CSR fast path holds) and no
//                       padding row gets more than ceil(n_pad / (n_cap - N))
//   labels [0, B)       copied
//   *n_valid = N        (the forward kernels skip rows >= N)
//   optional: a pack job -- one weight matrix (the layer-0 W_l) written in
//   ngnn_pack_weight's fragment order, so the captured step's forward reads
//   it prepacked (NGNN_WL_PREPACKED) instead of issuing a pack launch;
//   optional: the target-grouped CSR of the padded edges (rowptr int32
//   [n_cap + 1] by lower bound over the non-decreasing targets, col int32
//   [e_cap]), so the captured step needs no CSR-build launches; and the
//   dropout seed state advanced by one splitmix64 step (a fresh mask per
//   replay without a device RNG launch).
// Replaces the ~8 torch copy / arithmetic launches the slot load took.
// Requires target-sorted edges (NeighborLoader's order), as the CSR fast path.
#include "ngnn_internal.h"

namespace ngnn {
namespace {

// a source id as the consumers may read it: ids outside [0, N) (flagged
// NGNN_SLOT_RANGE) become row 0 (N >= 1 whenever there are edges to read)
__device__ __forceinline__ int64_t src_ok(int64_t s, int64_t N) { return (s >= 0 && s < N) ? s : 0; }

__global__ __launch_bounds__(256) void k_slot_load(
    const float *__restrict__ x, int64_t ldx, int64_t N, int64_t F, const int64_t *__restrict__ ei,
    int64_t ld_ei, int64_t E, const int64_t *__restrict__ y, int64_t B, float *__restrict__ sx,
    int64_t lds, int64_t n_cap, int64_t *__restrict__ sei, int64_t e_cap, int64_t *__restrict__ sy,
    int32_t *__restrict__ n_valid, int32_t *__restrict__ rowptr, int32_t *__restrict__ col,
    uint64_t *__restrict__ seed_state, const float **x_dev, int64_t *__restrict__ r_next,
    uint32_t gen, int32_t *__restrict__ n_edge_rows, const int64_t *xrow, const int64_t **xrow_dev,
    int32_t *__restrict__ colx, int vec, const float *__restrict__ pk_w, int64_t pk_ldw, int pk_fo,
    int pk_k, float *__restrict__ pk_dst, int32_t *err, const int32_t *__restrict__ cnt,
    uint64_t *__restrict__ gate) {
    if (cnt) {  // (ABI 19) the block's counts on the device; N / E: their bounds
        N = min(static_cast<int64_t>(cnt[0]), N);
        E = min(static_cast<int64_t>(cnt[1]), E);
    }
    const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
    if (x_dev) {  // zero-copy: the captured kernels read x where it is
        if (tid == 0) {
            *x_dev = x;
            // fused x[n_id]: x is the feature table, row r of the block is xrow[r]
            if (xrow_dev) *xrow_dev = xrow;
        }
    } else if (vec) {
        const int64_t f4 = F >> 2, total = N * f4;
        for (int64_t i = tid; i < total; i += nthr) {
            const int64_t r = i / f4, c = (i - r * f4) << 2;
            *reinterpret_cast<float4 *>(sx + r * lds + c) =
                *reinterpret_cast<const float4 *>(x + r * ldx + c);
        }
    } else {
        const int64_t total = N * F;
        for (int64_t i = tid; i < total; i += nthr) {
            const int64_t r = i / F, c = i - r * F;
            sx[r * lds + c] = x[r * ldx + c];
        }
    }
    const int64_t n_pad = e_cap - E, span = n_cap - N;
    int bad = 0;  // the block's contract: targets non-decreasing, ids in [0, N)
    for (int64_t e = tid; e < e_cap; e += nthr) {
        int64_t s, d;
        if (e < E) {
            s = ei[e];
            d = ei[ld_ei + e];
            if (s < 0 || s >= N || d < 0 || d >= N) bad |= NGNN_SLOT_RANGE;
            if (e > 0 && d < ei[ld_ei + e - 1]) bad |= NGNN_SLOT_UNSORTED;
            // (a contract-breaking block is trained on a wrong CSR, but never
            // out of bounds: a source outside [0, N) is read as row 0 by
            // every consumer -- gathers, scatters, the bounds below)
            s = src_ok(s, N);
        } else {
            d = N + ((e - E) * span) / n_pad;
            s = d;
        }
        if (sei) {
            sei[e] = s;
            sei[e_cap + e] = d;
        }
    }
    if (bad && err) atomicOr(err, bad);
    if (bad && gate)  // (this load's generation outranks every older load's bits)
        atomicMax(reinterpret_cast<unsigned long long *>(gate),
                  static_cast<unsigned long long>((static_cast<uint64_t>(gen) << 32) | static_cast<uint32_t>(bad)));
    for (int64_t i = tid; i < B; i += nthr) sy[i] = y[i];
    if (rowptr) {
        // rowptr[r] = first padded edge with target >= r.  Padding: closed
        // form (target of padding edge j is N + floor(j span / n_pad)); rows
        // past the last real target (NeighborLoader: every row that received
        // no edges, ~90% of a products block): E.
        // (a block breaking the contract gets a wrong CSR, but every write
        // stays inside rowptr: targets clamped to [-1, n_cap])
        const int64_t last_dst = E > 0 ? min(max(ei[ld_ei + E - 1], int64_t{-1}), n_cap) : -1;
        // rows up to the last target: edge e writes rowptr[r] = e for every
        // r in (dst[e-1], dst[e]] -- the lower bound of r over the sorted
        // targets, each row written once, two independent loads per edge
        // (a per-row binary search was a chain of ~17 dependent loads)
        for (int64_t e = tid; e < E; e += nthr) {
            const int64_t d = min(ei[ld_ei + e], n_cap);
            const int64_t p = e > 0 ? max(ei[ld_ei + e - 1], int64_t{-1}) : -1;
            for (int64_t r = p + 1; r <= d; ++r) rowptr[r] = static_cast<int32_t>(e);
        }
        for (int64_t r = last_dst + 1 + tid; r <= n_cap; r += nthr) {
            int64_t e;
            if (r <= N) {
                e = E;
            } else if (n_pad > 0) {
                e = E + min(n_pad, ((r - N) * n_pad + span - 1) / span);
            } else {
                e = E;
            }
            rowptr[r] = static_cast<int32_t>(r == n_cap ? e_cap : e);
        }
        for (int64_t e = tid; e < e_cap; e += nthr)
            col[e] = static_cast<int32_t>(e < E ? src_ok(ei[e], N) : N + ((e - E) * span) / n_pad);
    }
    if (colx) {
        // layer 0's gather columns: the sources' rows in the feature table
        // (padding edges feed skipped rows only: 0)
        for (int64_t e = tid; e < e_cap; e += nthr)
            colx[e] = static_cast<int32_t>((e < E && ei[e] >= 0 && ei[e] < N) ? (xrow ? xrow[ei[e]] : ei[e]) : 0);
    }
    if (r_next) {
        // max(B, 1 + max source over the edges into rows < B), as a 64-bit
        // atomicMax of (gen << 32 | value): this load's generation outranks
        // every stale value, so the word needs no reset launch; consumers
        // read its low 32 bits
        const uint64_t g = static_cast<uint64_t>(gen) << 32;
        uint64_t m = tid == 0 ? (g | static_cast<uint64_t>(B)) : 0;
        // (every edge looked at -- E <= the grid's threads on every NeighborLoader
        // block, so this is one edge per thread -- and no early exit: an
        // unsorted block still gets the bound of the edges it has)
        for (int64_t e = tid; e < E; e += nthr) {
            const int64_t d = ei[ld_ei + e];
            if (d >= 0 && d < B) m = max(m, g | static_cast<uint64_t>(src_ok(ei[e], N) + 1));
        }
        // one atomic per workgroup (same-address atomics serialise at the
        // memory side: one per wave was ~240 of them on a products block)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t other = (static_cast<uint64_t>(static_cast<uint32_t>(
                                        __shfl_xor(static_cast<int>(m >> 32), o))) << 32) |
                                   static_cast<uint32_t>(__shfl_xor(static_cast<int>(m), o));
            m = max(m, other);
        }
        __shared__ uint64_t s_m[4];  // (256 threads: 4 waves)
        if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            m = max(max(s_m[0], s_m[1]), max(s_m[2], s_m[3]));
            if (m) atomicMax(reinterpret_cast<unsigned long long *>(r_next), static_cast<unsigned long long>(m));
        }
    }
    if (pk_dst) {
        // pack job: pk_dst = ngnn_pack_weight(pk_w) -- the layout
        // [NT][KG][64 lanes][4]: lane l, element i of fragment (m, kg) holds
        // W[16 m + (l & 15)][16 kg + 4 (l >> 4) + i], zero outside Fo x K
        const int KG = (pk_k + 15) >> 4, NT = (pk_fo + 15) >> 4;
        const int64_t total = static_cast<int64_t>(NT) * KG * 256;
        for (int64_t i = tid; i < total; i += nthr) {
            const int64_t f = i >> 8;
            const int l = static_cast<int>((i >> 2) & 63), j = static_cast<int>(i & 3);
            const int m = static_cast<int>(f / KG), kg = static_cast<int>(f - static_cast<int64_t>(m) * KG);
            const int n = 16 * m + (l & 15), k = 16 * kg + 4 * (l >> 4) + j;
            pk_dst[i] = (n < pk_fo && k < pk_k) ? pk_w[static_cast<int64_t>(n) * pk_ldw + k] : 0.0f;
        }
    }
    if (tid == 0) {
        *n_valid = static_cast<int32_t>(N);
        if (n_edge_rows)  // rows past the last target have no in-edges
            *n_edge_rows = E > 0 ? static_cast<int32_t>(min(max(ei[ld_ei + E - 1] + 1, int64_t{0}), N)) : 0;
        if (seed_state) {  // splitmix64 step: state <- mix(state + golden gamma)
            uint64_t z = *seed_state + 0x9e3779b97f4a7c15ULL;
            z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
            z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
            *seed_state = z ^ (z >> 31);
        }
    }
}

}  // namespace
}  // namespace ngnn

using namespace ngnn;

extern "C" int ngnn_slot_load(const float *x, int64_t ldx, int64_t N, int64_t F,
                              const int64_t *edge_index, int64_t ld_ei, int64_t E, const int64_t *y,
                              int64_t B, float *slot_x, int64_t ld_slot, int64_t n_cap,
                              int64_t *slot_ei, int64_t e_cap, int64_t *slot_y, int32_t *n_valid,
                              int32_t *slot_rowptr, int32_t *slot_col, uint64_t *seed_state,
                              const float **x_dev, int64_t *r_next, uint32_t gen,
                              int32_t *n_edge_rows, const int64_t *xrow, const int64_t **xrow_dev,
                              int32_t *slot_colx, const float *pack_w, int64_t pack_ldw,
                              int64_t pack_fo, int64_t pack_k, float *pack_dst, int32_t *err,
                              const int32_t *counts_dev, uint64_t *gate, void *stream) {
    NGNN_RETURN_IF(N < 0 || F < 0 || E < 0 || B < 0 || (!slot_x && !x_dev) || !n_valid, NGNN_E_ARG);
    NGNN_RETURN_IF(!slot_ei && !slot_rowptr, NGNN_E_ARG);  // the edges must land somewhere
    NGNN_RETURN_IF(gate && !aligned(gate, 8), NGNN_E_ALIGN);
    NGNN_RETURN_IF(x_dev && (ldx != ld_slot || !aligned(x, 16)), NGNN_E_SHAPE);
    NGNN_RETURN_IF(xrow && (!x_dev || !xrow_dev), NGNN_E_ARG);  // indexed rows are zero-copy only
    NGNN_RETURN_IF((N > 0 && F > 0 && !x) || (E > 0 && !edge_index) || (B > 0 && (!y || !slot_y)),
                   NGNN_E_ARG);
    NGNN_RETURN_IF(ldx < F || ld_slot < F || ld_ei < E || (E > 0 && N == 0), NGNN_E_SHAPE);
    // padding needs rows to land on: at least one row past N when edges are padded
    NGNN_RETURN_IF(N > n_cap || E > e_cap || (E < e_cap && N >= n_cap), NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(N) || !fits_i32(n_cap) || !fits_i32(e_cap), NGNN_E_RANGE);
    NGNN_RETURN_IF((slot_rowptr == nullptr) != (slot_col == nullptr), NGNN_E_ARG);
    const int vec = (F % 4 == 0) && (ldx % 4 == 0) && (ld_slot % 4 == 0) && aligned(x, 16) &&
                    aligned(slot_x, 16);
    NGNN_RETURN_IF(pack_dst && (!pack_w || pack_fo <= 0 || pack_k <= 0 || pack_ldw < pack_k ||
                                !fits_i32(pack_fo) || !fits_i32(pack_k)), NGNN_E_ARG);
    const int64_t pack_n = pack_dst ? ceil_div(pack_fo, 16) * ceil_div(pack_k, 16) * 256 : 0;
    const int64_t work = std::max<int64_t>({x_dev ? 0 : N * F / 4, e_cap, n_cap + 1, B, pack_n, 1});
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>(ceil_div(work, 256), 4096));
    hipLaunchKernelGGL(k_slot_load, dim3(grid), dim3(256), 0, as_stream(stream), x, ldx, N, F,
                       edge_index, ld_ei, E, y, B, slot_x, ld_slot, n_cap, slot_ei, e_cap, slot_y,
                       n_valid, slot_rowptr, slot_col, seed_state, x_dev, r_next, gen, n_edge_rows,
                       xrow, xrow_dev, slot_colx, vec, pack_w, pack_ldw, static_cast<int>(pack_fo),
                       static_cast<int>(pack_k), pack_dst, err, counts_dev, gate);
    return launch_status();
}
