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
#include "ngnn_internal.h"

namespace ngnn {
namespace {

constexpr int kMaxFanout = 64;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
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
    const int64_t d = rowptr[v + 1] - b;
    int64_t *o = out_nbr + i * fanout;
    const int k = d < fanout ? static_cast<int>(d) : fanout;
    if (d <= fanout) {
        for (int j = 0; j < k; ++j) o[j] = gcol[b + j];
    } else {
        int64_t sel[kMaxFanout];
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
        for (int q = 0; q < k; ++q) o[q] = gcol[b + sel[q]];
    }
    for (int j = k; j < fanout; ++j) o[j] = -1;
    out_cnt[i] = k;
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
