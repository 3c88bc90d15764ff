// Adam for the training step (the reference's optimiser: torch.optim.Adam,
// model.py:66-69 [ext: torch]) as ONE launch over every parameter tensor:
// the last workgroup to finish (a device ticket) advances the step count,
// instead of torch's step increment + multi-tensor fused kernel.  Same update rule as torch Adam
// (amsgrad off, maximize off); bf16 parameters/gradients are widened, updated
// in fp32 against fp32 moments and rounded to nearest on store:
//   t = step + 1;  g += wd p;  m = m + (1 - b1)(g - m);  v = b2 v + (1 - b2) g^2
//   p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// The step count lives on the device (HIP-graph replays advance it).
#include <hip/hip_bf16.h>

#include "ngnn_internal.h"

namespace ngnn {
namespace {

constexpr int kMaxT = 16;

struct AdamTensors {
    float *p[kMaxT];  // fp32, or bf16 when bf[k] (update in fp32, stored rounded)
    const float *g[kMaxT];
    int bf[kMaxT];
    int vec[kMaxT];  // p, g, m, v aligned for 4-element vector accesses
    float *m[kMaxT];
    float *v[kMaxT];
    int64_t off[kMaxT + 1];  // prefix sums of numel
    int64_t boff[kMaxT + 1];  // prefix sums of virtual workgroups (ceil(numel / kAdamChunk))
    int n;
};

constexpr int kAdamTickets = 1024;            // uint32 words of the ticket (ABI 21; 64 before)
constexpr int kAdamTicketStride = 32;         // words between two group tickets: one 128-B line each
constexpr int kAdamGroups = kAdamTickets / kAdamTicketStride - 1;  // (line 0: the top ticket)
constexpr int kAdamVec = 4;                   // elements per thread
constexpr int kAdamChunk = 256 * kAdamVec;    // elements per virtual workgroup

__device__ __forceinline__ float bf16_bits_to_f(uint32_t b) { return __uint_as_float(b << 16); }
__device__ __forceinline__ uint32_t f_to_bf16_bits(float f) {  // RNE, NaN -> 0x7FC0
    const uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0u;
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// grid-stride over virtual workgroups of kAdamChunk elements (boff counts
// them per tensor): a few hundred workgroups, 16-B loads of 4 elements, and
// as many ticket atomics as workgroups (one per virtual workgroup serialised
// on the ticket's L2 channel: 40 us for Amazon-Computers' 1.6 M parameters)
__global__ __launch_bounds__(256) void k_adam(AdamTensors T, float *__restrict__ step,
                                              uint32_t *__restrict__ ticket, float lr, float b1,
                                              float b2, float eps, float wd, const uint64_t *gate,
                                              const int64_t *gate_gen) {
    if (slot_gated(gate, gate_gen)) return;  // (a contract-breaking block: no update, no step; ABI 20)
    const float t = *step + 1.0f;
    // the completion ticket is taken right after every thread has read the
    // count (what it guards), not after the update: the atomic's round trip
    // overlaps the workgroup's loads instead of holding its end (a ticket at
    // the end measured 12.4 vs 8.5 us for update + increment launches on
    // Amazon-Computers' 0.8 M parameters, tools/adam_micro.py)
    const unsigned gi = blockIdx.x >> 5, gs = min(32u, gridDim.x - (gi << 5));
    uint32_t tk = 0u;
    if (ticket) {
        asm volatile("" ::"v"(t));  // (this thread's read of *step has landed)
        __syncthreads();
        if (threadIdx.x == 0) tk = atomicAdd(ticket + kAdamTicketStride * (1 + gi), 1u);
    }
    const float bc1 = 1.0f - powf(b1, t);
    const float bc2s = sqrtf(1.0f - powf(b2, t));
    const float step_size = lr / bc1;
    auto upd = [&](float g, float &p, float &m, float &v) {
        if (wd != 0.0f) g = g + wd * p;
        m = m + (1.0f - b1) * (g - m);
        v = b2 * v + (1.0f - b2) * g * g;
        const float denom = sqrtf(v) / bc2s + eps;
        p = p - step_size * (m / denom);
    };
    const int64_t nvb = T.boff[T.n];
    // one virtual workgroup's operands, loaded a workgroup-stride ahead of its
    // update: the next one's loads are in flight while this one computes and
    // stores (distinct elements: a load issued before a store to other
    // addresses returns what it would alone)
    struct Ld {
        int k;
        int64_t j, n;
        bool vec;
        float4 m4, v4;
        float g[4], p[4];
    };
    auto load = [&](int64_t vb, int &k, Ld &L) __attribute__((always_inline)) {
        // virtual workgroup -> tensor: uniform (scalar loads of its pointers)
        while (k + 1 < T.n && vb >= T.boff[k + 1]) ++k;
        L.k = k;
        L.n = T.off[k + 1] - T.off[k];
        L.j = (vb - T.boff[k]) * kAdamChunk + threadIdx.x * kAdamVec;
        L.vec = T.vec[k] && L.j + kAdamVec <= L.n;
        if (!L.vec) return;  // (the tensor's ragged tail or an unaligned view: at the update)
        const int64_t j = L.j;
        L.m4 = *reinterpret_cast<const float4 *>(T.m[k] + j);
        L.v4 = *reinterpret_cast<const float4 *>(T.v[k] + j);
        if (T.bf[k]) {  // bf16 parameter and gradient: widen (exact), update, round
            const uint2 gb = *reinterpret_cast<const uint2 *>(reinterpret_cast<const uint16_t *>(T.g[k]) + j);
            const uint2 pb = *reinterpret_cast<const uint2 *>(reinterpret_cast<const uint16_t *>(T.p[k]) + j);
            L.g[0] = bf16_bits_to_f(gb.x & 0xffffu); L.g[1] = bf16_bits_to_f(gb.x >> 16);
            L.g[2] = bf16_bits_to_f(gb.y & 0xffffu); L.g[3] = bf16_bits_to_f(gb.y >> 16);
            L.p[0] = bf16_bits_to_f(pb.x & 0xffffu); L.p[1] = bf16_bits_to_f(pb.x >> 16);
            L.p[2] = bf16_bits_to_f(pb.y & 0xffffu); L.p[3] = bf16_bits_to_f(pb.y >> 16);
        } else {
            const float4 g4 = *reinterpret_cast<const float4 *>(T.g[k] + j);
            const float4 p4 = *reinterpret_cast<const float4 *>(T.p[k] + j);
            L.g[0] = g4.x; L.g[1] = g4.y; L.g[2] = g4.z; L.g[3] = g4.w;
            L.p[0] = p4.x; L.p[1] = p4.y; L.p[2] = p4.z; L.p[3] = p4.w;
        }
    };
    auto apply = [&](Ld &L) __attribute__((always_inline)) {
        const int k = L.k;
        const int64_t j = L.j, n = L.n;
        if (j >= n) return;
        if (L.vec) {
            upd(L.g[0], L.p[0], L.m4.x, L.v4.x);
            upd(L.g[1], L.p[1], L.m4.y, L.v4.y);
            upd(L.g[2], L.p[2], L.m4.z, L.v4.z);
            upd(L.g[3], L.p[3], L.m4.w, L.v4.w);
            *reinterpret_cast<float4 *>(T.m[k] + j) = L.m4;
            *reinterpret_cast<float4 *>(T.v[k] + j) = L.v4;
            if (T.bf[k]) {
                const uint2 o{f_to_bf16_bits(L.p[0]) | (f_to_bf16_bits(L.p[1]) << 16),
                              f_to_bf16_bits(L.p[2]) | (f_to_bf16_bits(L.p[3]) << 16)};
                *reinterpret_cast<uint2 *>(reinterpret_cast<uint16_t *>(T.p[k]) + j) = o;
            } else {
                *reinterpret_cast<float4 *>(T.p[k] + j) = float4{L.p[0], L.p[1], L.p[2], L.p[3]};
            }
            return;
        }
        for (int64_t e = j; e < min(j + kAdamVec, n); ++e) {
            float g, p;
            if (T.bf[k]) {
                g = bf16_bits_to_f(reinterpret_cast<const uint16_t *>(T.g[k])[e]);
                p = bf16_bits_to_f(reinterpret_cast<const uint16_t *>(T.p[k])[e]);
            } else {
                g = T.g[k][e];
                p = T.p[k][e];
            }
            float m = T.m[k][e], v = T.v[k][e];
            upd(g, p, m, v);
            T.m[k][e] = m;
            T.v[k][e] = v;
            if (T.bf[k]) reinterpret_cast<uint16_t *>(T.p[k])[e] = static_cast<uint16_t>(f_to_bf16_bits(p));
            else T.p[k][e] = p;
        }
    };
    int k = 0;
    int64_t vb = blockIdx.x;
    if (vb < nvb) {
        Ld cur;
        load(vb, k, cur);
        for (;;) {
            const int64_t nx = vb + gridDim.x;
            if (nx >= nvb) {
                apply(cur);
                break;
            }
            Ld nl;
            load(nx, k, nl);
            apply(cur);
            cur = nl;
            vb = nx;
        }
    }
    if (ticket && threadIdx.x == 0 && tk == gs - 1) {
        // the last of its group of 32 (every member has read *step): counts on
        // the top ticket (two levels, ABI 17 -- same-address atomics
        // serialise at the memory side); the last group advances the count
        ticket[kAdamTicketStride * (1 + gi)] = 0u;
        const unsigned ngr = (gridDim.x + 31) >> 5;
        if (atomicAdd(ticket, 1u) == ngr - 1) {
            *step = t;
            *ticket = 0u;
        }
    }
}

__global__ void k_step_inc(float *step, const uint64_t *gate, const int64_t *gate_gen) {
    if (!slot_gated(gate, gate_gen)) *step += 1.0f;
}

}  // namespace
}  // namespace ngnn

using namespace ngnn;

extern "C" int ngnn_adam_step(int n_tensors, float *const *params, const float *const *grads,
                              float *const *exp_avgs, float *const *exp_avg_sqs,
                              const int64_t *numels, const int32_t *dtypes, float *step,
                              uint32_t *ticket, float lr,
                              float beta1, float beta2, float eps, float weight_decay,
                              const uint64_t *gate, const int64_t *gate_gen, void *stream) {
    NGNN_RETURN_IF(n_tensors < 0 || !step, NGNN_E_ARG);
    NGNN_RETURN_IF(n_tensors > 0 && (!params || !grads || !exp_avgs || !exp_avg_sqs || !numels),
                   NGNN_E_ARG);
    hipStream_t st = as_stream(stream);
    // the ticket path needs every tensor in one launch (one reader set of *step)
    if (n_tensors > kMaxT) ticket = nullptr;
    static const bool no_ticket = [] {  // (NGNN_ADAM_NO_TICKET=1, read once: update + increment launches -- A/B)
        const char *e = std::getenv("NGNN_ADAM_NO_TICKET");
        return e && e[0] == '1';
    }();
    if (no_ticket) ticket = nullptr;
    bool launched = false;
    for (int base = 0; base < n_tensors; base += kMaxT) {
        AdamTensors T;
        T.n = std::min(kMaxT, n_tensors - base);
        T.off[0] = 0;
        for (int k = 0; k < T.n; ++k) {
            NGNN_RETURN_IF(numels[base + k] < 0, NGNN_E_ARG);
            NGNN_RETURN_IF(numels[base + k] > 0 && (!params[base + k] || !grads[base + k] ||
                                                    !exp_avgs[base + k] || !exp_avg_sqs[base + k]),
                           NGNN_E_ARG);
            T.p[k] = params[base + k];
            T.g[k] = grads[base + k];
            T.m[k] = exp_avgs[base + k];
            T.bf[k] = dtypes ? (dtypes[base + k] == NGNN_BF16) : 0;
            NGNN_RETURN_IF(dtypes && dtypes[base + k] != NGNN_F32 && dtypes[base + k] != NGNN_BF16,
                           NGNN_E_DTYPE);
            T.v[k] = exp_avg_sqs[base + k];
            const size_t pa = T.bf[k] ? 8 : 16;  // 4 elements of p and g
            T.vec[k] = aligned(T.p[k], pa) && aligned(T.g[k], pa) && aligned(T.m[k], 16) &&
                       aligned(T.v[k], 16);
            T.off[k + 1] = T.off[k] + numels[base + k];
        }
        if (T.off[T.n] == 0) continue;
        T.boff[0] = 0;
        for (int k = 0; k < T.n; ++k) T.boff[k + 1] = T.boff[k] + ceil_div(numels[base + k], kAdamChunk);
        NGNN_RETURN_IF(T.boff[T.n] > (int64_t{1} << 31) - 1, NGNN_E_RANGE);
        // (without the ticket -- NGNN_ADAM_NO_TICKET=1 -- the update is a
        // separate launch from the one-lane increment: on Amazon-Computers'
        // 0.8 M parameters 8.6 vs 11.9 us per step in a graph of Adam steps
        // alone (tools/adam_micro.py), but 9.3 + 4.0 vs 12.8 us inside the
        // training step's graph: the ticket stays)
        // at most 2 workgroups per CU: the rest is the grid-stride loop (and at
        // most 32 x kAdamGroups -- the ticket's groups)
        // (NGNN_ADAM_WG_PER_CU, read once: the per-CU cap -- A/B)
        static const int wg_cu = [] {
            const char *e = std::getenv("NGNN_ADAM_WG_PER_CU");
            return e ? std::max(1, std::atoi(e)) : 2;
        }();
        const unsigned grid = static_cast<unsigned>(std::min<int64_t>(std::min<int64_t>(T.boff[T.n], wg_cu * num_cus()),
                                                                      32 * kAdamGroups));
        hipLaunchKernelGGL(k_adam, dim3(grid), dim3(256), 0, st, T, step, ticket, lr, beta1, beta2,
                           eps, weight_decay, gate, gate_gen);
        const int rc = launch_status();
        if (rc) return rc;
        launched = true;
    }
    if (ticket && launched) return NGNN_OK;
    hipLaunchKernelGGL(k_step_inc, dim3(1), dim3(1), 0, st, step, gate, gate_gen);
    return launch_status();
}

// ---- fp32 -> bf16 rows (a bf16 model's logits): round to nearest even, every
// NaN to the canonical quiet NaN 0x7FC0 (c10::BFloat16's round_to_nearest_even,
// which torch's device cast uses); 4 values per thread, grid-stride.  Replaces
// Tensor.to(torch.bfloat16) on the [N, C] logits.
namespace ngnn {
namespace {
// W8: 8 elements per thread step (two 16-B loads, one 16-B store: wide
// stores move the logits of a 1.5 M-row block at twice the 8-B stores' rate);
// else 4 (8-B stores, dst only 8-B aligned)
template <bool W8>
__global__ __launch_bounds__(256) void k_cast_bf16(const float *__restrict__ src,
                                                    uint16_t *__restrict__ dst, int64_t n,
                                                    const int32_t *__restrict__ rows_dev, int64_t row_elems) {
    // (rows_dev: only the block's real rows -- a graph slot's logits are
    // sized for its capacity, 2.3x the rows of a 3-layer products block)
    if (rows_dev) n = min(n, static_cast<int64_t>(max(*rows_dev, 0)) * row_elems);
    auto rne = [](float f) -> uint32_t {
        const uint32_t u = __float_as_uint(f);
        if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0u;
        return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
    };
    auto pack = [&](float4 v) { return uint2{rne(v.x) | (rne(v.y) << 16), rne(v.z) | (rne(v.w) << 16)}; };
    constexpr int E = W8 ? 8 : 4;
    const int64_t nv = n / E;
    const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
    int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
    // U steps' loads in flight per thread before the first store
    constexpr int U = W8 ? 2 : 4;
    auto step_load = [&](int64_t k, float4 (&v)[2]) {
        v[0] = reinterpret_cast<const float4 *>(src)[k * (E / 4)];
        if (W8) v[1] = reinterpret_cast<const float4 *>(src)[k * 2 + 1];
    };
    auto step_store = [&](int64_t k, const float4 (&v)[2]) {
        if (W8) {
            const uint2 a = pack(v[0]), b = pack(v[1]);
            reinterpret_cast<uint4 *>(dst)[k] = uint4{a.x, a.y, b.x, b.y};
        } else {
            reinterpret_cast<uint2 *>(dst)[k] = pack(v[0]);
        }
    };
    for (; i + (U - 1) * stride < nv; i += U * stride) {
        float4 v[U][2];
#pragma unroll
        for (int u = 0; u < U; ++u) step_load(i + u * stride, v[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) step_store(i + u * stride, v[u]);
    }
    for (; i < nv; i += stride) {
        float4 v[2];
        step_load(i, v);
        step_store(i, v);
    }
    for (int64_t k = E * nv + blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; k < n; k += stride)
        dst[k] = static_cast<uint16_t>(rne(src[k]));
}
}  // namespace
}  // namespace ngnn

static int cast_f32_bf16(const float *src, void *dst, int64_t n, const int32_t *rows_dev, int64_t row_elems,
                         void *stream) {
    using namespace ngnn;
    NGNN_RETURN_IF(n < 0 || (n > 0 && (!src || !dst)), NGNN_E_ARG);
    NGNN_RETURN_IF(!aligned(src, 16) || !aligned(dst, 8), NGNN_E_SHAPE);
    if (n == 0) return NGNN_OK;
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>(ceil_div(ceil_div(n, 8), 256), 2048));
    if (aligned(dst, 16))
        hipLaunchKernelGGL(k_cast_bf16<true>, dim3(grid), dim3(256), 0, as_stream(stream), src,
                           static_cast<uint16_t *>(dst), n, rows_dev, row_elems);
    else
        hipLaunchKernelGGL(k_cast_bf16<false>, dim3(grid), dim3(256), 0, as_stream(stream), src,
                           static_cast<uint16_t *>(dst), n, rows_dev, row_elems);
    return launch_status();
}

extern "C" int ngnn_cast_f32_bf16(const float *src, void *dst, int64_t n, void *stream) {
    return cast_f32_bf16(src, dst, n, nullptr, 0, stream);
}

extern "C" int ngnn_cast_f32_bf16_rows(const float *src, void *dst, int64_t n_rows, int64_t row_elems,
                                       const int32_t *n_rows_dev, void *stream) {
    NGNN_RETURN_IF(n_rows < 0 || row_elems < 0, NGNN_E_ARG);
    return cast_f32_bf16(src, dst, n_rows * row_elems, n_rows_dev, row_elems, stream);
}

// ---- n tensors cast in ONE launch: bf16 -> fp32 (exact) or fp32 -> bf16
// (round to nearest even, NaN kept): a bf16 model's parameters widened for
// the fused kernels and their fp32 gradients narrowed back (each was an ATen
// copy kernel per tensor)
namespace ngnn {
namespace {
struct CastTensors {
    const void *src[kMaxT];
    void *dst[kMaxT];
    int64_t off[kMaxT + 1];  // prefix sums of numel
    int n;
};
template <bool TO_BF16>
__global__ __launch_bounds__(256) void k_cast_tensors(CastTensors T) {
    const int64_t total = T.off[T.n];
    const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total; i += stride) {
        int k = 0;
        while (i >= T.off[k + 1]) ++k;  // (<= 16 tensors)
        const int64_t j = i - T.off[k];
        if (TO_BF16) {
            const float v = static_cast<const float *>(T.src[k])[j];
            static_cast<__bf16 *>(T.dst[k])[j] = static_cast<__bf16>(v);
        } else {
            const uint16_t b = static_cast<const uint16_t *>(T.src[k])[j];
            static_cast<float *>(T.dst[k])[j] = __uint_as_float(static_cast<uint32_t>(b) << 16);
        }
    }
}
}  // namespace
}  // namespace ngnn

extern "C" int ngnn_cast_tensors(int n, const void *const *src, void *const *dst, const int64_t *numels,
                                 int to_bf16, void *stream) {
    using namespace ngnn;
    NGNN_RETURN_IF(n < 0 || n > kMaxT || (n > 0 && (!src || !dst || !numels)), NGNN_E_ARG);
    CastTensors T;
    T.n = n;
    T.off[0] = 0;
    for (int k = 0; k < n; ++k) {
        NGNN_RETURN_IF(numels[k] < 0 || (numels[k] > 0 && (!src[k] || !dst[k])), NGNN_E_ARG);
        T.src[k] = src[k];
        T.dst[k] = dst[k];
        T.off[k + 1] = T.off[k] + numels[k];
    }
    if (n == 0 || T.off[n] == 0) return NGNN_OK;
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>(ceil_div(T.off[n], 256), 1024));
    if (to_bf16) hipLaunchKernelGGL(k_cast_tensors<true>, dim3(grid), dim3(256), 0, as_stream(stream), T);
    else hipLaunchKernelGGL(k_cast_tensors<false>, dim3(grid), dim3(256), 0, as_stream(stream), T);
    return launch_status();
}

// ---- n tensors of mixed dtypes copied / cast and divided in ONE launch (ABI
// 18): the data-parallel gradient bucket's pack (bf16 or fp32 gradients ->
// the fp32 bucket) and unpack (bucket / world -> the gradients, in place for
// the fp32 ones that ARE bucket views).  The division is the IEEE quotient,
// as Tensor.div_ computes it; divisor 1 skips it (exact).
namespace ngnn {
namespace {
struct CastTensorsEx {
    const void *src[kMaxT];
    void *dst[kMaxT];
    int64_t off[kMaxT + 1];
    uint32_t sbf, dbf;  // bit k: tensor k's source / destination is bf16
    int n;
    float div;
};
__global__ __launch_bounds__(256) void k_cast_tensors_ex(CastTensorsEx T) {
    const int64_t total = T.off[T.n];
    const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total; i += stride) {
        int k = 0;
        while (i >= T.off[k + 1]) ++k;  // (<= 16 tensors)
        const int64_t j = i - T.off[k];
        float v = (T.sbf >> k) & 1u
                      ? __uint_as_float(static_cast<uint32_t>(static_cast<const uint16_t *>(T.src[k])[j]) << 16)
                      : static_cast<const float *>(T.src[k])[j];
        if (T.div != 1.0f) v = v / T.div;
        if ((T.dbf >> k) & 1u) static_cast<__bf16 *>(T.dst[k])[j] = static_cast<__bf16>(v);
        else static_cast<float *>(T.dst[k])[j] = v;
    }
}
}  // namespace
}  // namespace ngnn

extern "C" int ngnn_cast_tensors_ex(int n, const void *const *src, void *const *dst, const int64_t *numels,
                                    const int32_t *src_dtypes, const int32_t *dst_dtypes, float divisor,
                                    void *stream) {
    using namespace ngnn;
    NGNN_RETURN_IF(n < 0 || n > kMaxT || (n > 0 && (!src || !dst || !numels || !src_dtypes || !dst_dtypes)),
                   NGNN_E_ARG);
    NGNN_RETURN_IF(!(divisor != 0.0f), NGNN_E_ARG);
    CastTensorsEx T;
    T.n = n;
    T.off[0] = 0;
    T.sbf = T.dbf = 0;
    T.div = divisor;
    for (int k = 0; k < n; ++k) {
        NGNN_RETURN_IF(numels[k] < 0 || (numels[k] > 0 && (!src[k] || !dst[k])), NGNN_E_ARG);
        NGNN_RETURN_IF((src_dtypes[k] != NGNN_F32 && src_dtypes[k] != NGNN_BF16) ||
                           (dst_dtypes[k] != NGNN_F32 && dst_dtypes[k] != NGNN_BF16),
                       NGNN_E_DTYPE);
        // (in place only without a width change)
        NGNN_RETURN_IF(src[k] == dst[k] && src_dtypes[k] != dst_dtypes[k], NGNN_E_ARG);
        T.src[k] = src[k];
        T.dst[k] = dst[k];
        T.off[k + 1] = T.off[k] + numels[k];
        T.sbf |= static_cast<uint32_t>(src_dtypes[k] == NGNN_BF16) << k;
        T.dbf |= static_cast<uint32_t>(dst_dtypes[k] == NGNN_BF16) << k;
    }
    if (n == 0 || T.off[n] == 0) return NGNN_OK;
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>(ceil_div(T.off[n], 256), 1024));
    hipLaunchKernelGGL(k_cast_tensors_ex, dim3(grid), dim3(256), 0, as_stream(stream), T);
    return launch_status();
}

// ---- bf16 rows -> fp32 rows [0, min(n_rows, *n_rows_dev)) x F (a bf16 model's
// activations widened for the backward kernels that read fp32 masks, rows
// below a device-side bound only); exact.
namespace ngnn {
namespace {
__global__ __launch_bounds__(256) void k_widen_bf16_rows(const uint16_t *__restrict__ src, int64_t lds,
                                                         int F, int n_rows,
                                                         const int32_t *__restrict__ n_rows_dev,
                                                         float *__restrict__ dst, int64_t ldd) {
    int rows = n_rows;
    if (n_rows_dev) rows = min(rows, *n_rows_dev);
    const int64_t total = static_cast<int64_t>(rows) * F;
    const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
    for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total; i += stride) {
        const int64_t r = i / F;
        const int c = static_cast<int>(i - r * F);
        dst[r * ldd + c] = __uint_as_float(static_cast<uint32_t>(src[r * lds + c]) << 16);
    }
}
}  // namespace
}  // namespace ngnn

extern "C" int ngnn_widen_bf16_rows(const void *src, int64_t lds, int64_t F, int64_t n_rows,
                                    const int32_t *n_rows_dev, float *dst, int64_t ldd,
                                    void *stream) {
    using namespace ngnn;
    NGNN_RETURN_IF(F < 0 || n_rows < 0 || lds < F || ldd < F, NGNN_E_ARG);
    NGNN_RETURN_IF(!fits_i32(F) || !fits_i32(n_rows), NGNN_E_RANGE);
    if (F == 0 || n_rows == 0) return NGNN_OK;
    NGNN_RETURN_IF(!src || !dst, NGNN_E_ARG);
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>(ceil_div(n_rows * F, 256), 4096));
    hipLaunchKernelGGL(k_widen_bf16_rows, dim3(grid), dim3(256), 0, as_stream(stream),
                       static_cast<const uint16_t *>(src), lds, static_cast<int>(F),
                       static_cast<int>(n_rows), n_rows_dev, dst, ldd);
    return launch_status();
}
