// Seed-row cross entropy for the training step: the loss the reference's
// loop takes on the first batch_size rows of the SAGE output
// (pipeline.py:158, F.cross_entropy(out[:batch_size], y[:batch_size])
// [ext: torch]), as two launches instead of the ~9 of softmax / nll /
// slice-backward / fills.
//
// forward : loss = sum_{r<B, y_r != ignore} (lse(x_r) - x_r[y_r]) / #valid
//           one wave per row, then one workgroup adds the row losses in a
//           fixed order (second launch) -> deterministic.
// backward: d x_r[c] = g (softmax(x_r)[c] - [c == y_r]) / #valid for r < B,
//           0 for ignored rows; rows >= B are not written (the caller keeps
//           them zero).  One wave per row.
#include "ngnn_internal.h"

namespace ngnn {
namespace {

// the one-launch forward + gradient recounts the labels per workgroup
// (B^2 / 4 reads): above this many seed rows the O(B) three-launch path
constexpr int64_t kXentFusedMaxB = 4096;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ float wave_maxf(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

// log-sum-exp of one row (torch's log_softmax order: max, then sum of
// exp(x - max)); a NaN anywhere makes the sum NaN
__device__ __forceinline__ float row_lse(const float *__restrict__ xr, int C, int lane) {
    float m = -INFINITY;
    for (int c = lane; c < C; c += 64) m = fmaxf(m, xr[c]);
    m = wave_maxf(m);
    float s = 0.0f;
    for (int c = lane; c < C; c += 64) s += expf(xr[c] - m);
    s = wave_sum(s);
    return m + logf(s);
}

// one wave per row: ws[r] = row loss (0 if ignored), ws[B + r] = 1/0 valid
__global__ __launch_bounds__(256) void k_xent_rows(const float *__restrict__ x, int64_t ld, int B,
                                                   int C, const int64_t *__restrict__ y,
                                                   int64_t ignore, float *__restrict__ ws) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= B) return;
    const int64_t t = y[r];
    float l = 0.0f, v = 0.0f;
    if (t != ignore) {
        const float *xr = x + static_cast<int64_t>(r) * ld;
        const float lse = row_lse(xr, C, lane);
        l = (t >= 0 && t < C) ? lse - xr[t] : NAN;  // out-of-range label: NaN, no OOB read
        v = 1.0f;
    }
    if (lane == 0) {
        ws[r] = l;
        ws[B + r] = v;
    }
}

// one workgroup adds the row losses in a fixed order (strided per thread,
// then a fixed tree) -> deterministic; a separate launch, so no cross-XCD
// fences or tickets are needed
__global__ __launch_bounds__(256) void k_xent_sum(const float *__restrict__ ws, int B,
                                                  float *__restrict__ loss,
                                                  float *__restrict__ count) {
    float s = 0.0f, n = 0.0f;
    for (int i = threadIdx.x; i < B; i += 256) {
        s += ws[i];
        n += ws[B + i];
    }
    __shared__ float ss[256], sn[256];
    ss[threadIdx.x] = s;
    sn[threadIdx.x] = n;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if (threadIdx.x < h) {
            ss[threadIdx.x] += ss[threadIdx.x + h];
            sn[threadIdx.x] += sn[threadIdx.x + h];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        *loss = ss[0] / sn[0];  // 0/0 = NaN when every row is ignored, as torch
        *count = sn[0];
    }
}

__global__ __launch_bounds__(256) void k_xent_bwd(const float *__restrict__ x, int64_t ld, int B,
                                                  int C, const int64_t *__restrict__ y,
                                                  int64_t ignore, const float *__restrict__ ws,
                                                  const float *__restrict__ g,
                                                  const float *__restrict__ count,
                                                  float *__restrict__ dx, int64_t ldd) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= B) return;
    const float *xr = x + static_cast<int64_t>(r) * ld;
    float *dr = dx + static_cast<int64_t>(r) * ldd;
    const int64_t t = y[r];
    if (t == ignore) {
        for (int c = lane; c < C; c += 64) dr[c] = 0.0f;
        return;
    }
    // recomputed rather than read back from ws: another forward on the same
    // workspace (two losses per step, co-teaching) may have overwritten it
    (void)ws;
    const float lse = row_lse(xr, C, lane);
    const float scale = (g ? *g : 1.0f) / *count;  // (g NULL: the unit scale of loss.backward())
    for (int c = lane; c < C; c += 64) {
        const float p = expf(xr[c] - lse);
        dr[c] = scale * (p - (c == t ? 1.0f : 0.0f));
    }
}

// forward AND the unit-scale gradient in ONE launch (the training step's
// loss.backward(1) needs nothing else): every workgroup counts the valid
// labels of y[0..B) itself (B int64 reads from L2: no count pass), each wave
// takes one row -- its loss and its gradient row (softmax - onehot) / count
// (zeros for an ignored row) -- the workgroup adds its rows' losses in wave
// order, and the LAST workgroup to finish (a device ticket) adds the
// workgroup sums in a fixed order: loss = sum / count, deterministic.
// ws: partial sums [gridDim.x] floats; ticket (uint32, zero between calls).
// Every workgroup reads all B labels, so the count costs B^2 / 4 label reads
// in all: the host takes this kernel only for B <= kXentFusedMaxB (the
// training step's seed rows) and the three-launch O(B) path above it.
// The hand-off is the measured gfx950 form of MI355X_MICROARCH.md ("Valid
// forms", first table row): every partial an agent-scope (sc1) store drained
// by s_waitcnt vmcnt(0) before ONE agent-scope atomic add per workgroup, the
// last adder reads every partial with agent-scope (sc1) loads.  It leans on
// gfx9's vmcnt counting stores and on sc1 codegen, hence the target check.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "k_xent_fused's fence-free hand-off is verified for gfx950 only"
#endif
__global__ __launch_bounds__(256) void k_xent_fused(const float *__restrict__ x, int64_t ld, int B,
                                                    int C, const int64_t *__restrict__ y,
                                                    int64_t ignore, float *__restrict__ part,
                                                    uint32_t *__restrict__ ticket,
                                                    float *__restrict__ loss,
                                                    float *__restrict__ count,
                                                    float *__restrict__ dx, int64_t ldd) {
    __shared__ float s_red[256];
    __shared__ float s_row[4];
    __shared__ int s_last;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float nv = 0.0f;
    for (int i = threadIdx.x; i < B; i += 256) nv += (y[i] != ignore) ? 1.0f : 0.0f;
    s_red[threadIdx.x] = nv;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if (threadIdx.x < h) s_red[threadIdx.x] += s_red[threadIdx.x + h];
        __syncthreads();
    }
    const float cnt = s_red[0];
    const int r = blockIdx.x * 4 + wv;
    float l = 0.0f;
    if (r < B) {
        const float *xr = x + static_cast<int64_t>(r) * ld;
        float *dr = dx + static_cast<int64_t>(r) * ldd;
        const int64_t t = y[r];
        if (t == ignore) {
            for (int c = lane; c < C; c += 64) dr[c] = 0.0f;
        } else {
            const float lse = row_lse(xr, C, lane);
            l = (t >= 0 && t < C) ? lse - xr[t] : NAN;  // out-of-range label: NaN, no OOB read
            for (int c = lane; c < C; c += 64)
                dr[c] = (expf(xr[c] - lse) - (c == t ? 1.0f : 0.0f)) / cnt;
        }
    }
    if (lane == 0) s_row[wv] = l;
    __syncthreads();
    if (threadIdx.x == 0) {
        // hand-off without fences (MI355X_MICROARCH.md, inter-workgroup
        // visibility): the partial goes out as an agent-scope (sc1,
        // write-through) store, drained before the ticket; the last workgroup
        // reads every partial with agent-scope (sc1) loads.  (An agent fence
        // pair -- L2 write-back + invalidate -- cost ~10 us here.)
        __hip_atomic_store(part + blockIdx.x, ((s_row[0] + s_row[1]) + s_row[2]) + s_row[3],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_last = atomicAdd(ticket, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!s_last) return;
    float s = 0.0f;
    for (int i = threadIdx.x; i < static_cast<int>(gridDim.x); i += 256)
        s += __hip_atomic_load(part + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_red[threadIdx.x] = s;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if (threadIdx.x < h) s_red[threadIdx.x] += s_red[threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        *loss = s_red[0] / cnt;  // 0/0 = NaN when every row is ignored, as torch
        *count = cnt;
        *ticket = 0u;
    }
}

// ---------------------------------------------------------------------------
// Co-teaching loss (CTLoss.forward, losses.py:19-49) on the device.  The
// reference takes each model's per-row cross entropy, np.argsort's it on the
// host (two device->host syncs per batch), keeps the num_remember smallest
// rows of each model and trains each model on the rows the OTHER model kept.
//
// ws (floats): l[2][B] row losses, v[2][B] valid flags, sel[2][B] "row gets
// gradient" flags, cnt[2] selected valid rows per model.
// Sort order: ascending loss, ties by row index (np.argsort's default
// quicksort leaves tie order unspecified; NaN sorts last, as numpy).

constexpr int kCtMaxB = 8192;  // bitonic sort of 64-bit keys in 64 KiB of LDS

__global__ __launch_bounds__(256) void k_ct_rows(const float *__restrict__ y1, int64_t ld1,
                                                 const float *__restrict__ y2, int64_t ld2, int B,
                                                 int C, const int64_t *__restrict__ t,
                                                 int64_t ignore, float *__restrict__ ws) {
    const int lane = threadIdx.x & 63;
    const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (g >= 2 * B) return;
    const int m = g >= B, r = g - m * B;
    const float *xr = (m ? y2 : y1) + static_cast<int64_t>(r) * (m ? ld2 : ld1);
    const int64_t c = t[r];
    float l = 0.0f, v = 0.0f;
    if (c != ignore) {
        const float lse = row_lse(xr, C, lane);
        l = (c >= 0 && c < C) ? lse - xr[c] : NAN;
        v = 1.0f;
    }
    if (lane == 0) {
        ws[m * B + r] = l;
        ws[2 * B + m * B + r] = v;
    }
}

__device__ __forceinline__ uint32_t order_key(float f) {
    if (f != f) return 0xffffffffu;  // NaN last
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// workgroup m sorts model m's row losses; selects, for the OTHER model o,
// the rows model m keeps: loss_o = mean CE of model o over them; pure_m =
// mean noise_or_not[ind[kept_m]]
__global__ __launch_bounds__(1024) void k_ct_select(float *__restrict__ ws, int B, int R,
                                                    const int64_t *__restrict__ ind,
                                                    const uint8_t *__restrict__ clean,
                                                    int64_t n_clean, int64_t *__restrict__ ind1,
                                                    int64_t *__restrict__ ind2,
                                                    float *__restrict__ out,
                                                    int *__restrict__ err) {
    __shared__ uint64_t key[kCtMaxB];
    __shared__ float rs[1024], rc[1024], rp[1024];
    const int m = blockIdx.x, o = 1 - m, tid = threadIdx.x;
    int P = 1;
    while (P < B) P <<= 1;
    const float *l = ws + m * B;
    for (int i = tid; i < P; i += 1024)
        key[i] = i < B ? (static_cast<uint64_t>(order_key(l[i])) << 32) | static_cast<uint32_t>(i)
                       : ~0ull;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < P; i += 1024) {
                const int p = i ^ j;
                if (p > i) {
                    const uint64_t a = key[i], b = key[p];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) {
                        key[i] = b;
                        key[p] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
    int64_t *im = m ? ind2 : ind1;
    for (int i = tid; i < B; i += 1024) im[i] = static_cast<int64_t>(key[i] & 0xffffffffu);
    float *sel = ws + 4 * B + o * B;  // rows of model o that receive gradient
    for (int i = tid; i < B; i += 1024) sel[i] = 0.0f;
    __syncthreads();
    const float *lo = ws + o * B, *vo = ws + 2 * B + o * B;
    float s = 0.0f, c = 0.0f, p = 0.0f;
    int bad = 0;
    for (int j = tid; j < R; j += 1024) {
        const int r = static_cast<int>(key[j] & 0xffffffffu);
        sel[r] = 1.0f;
        s += lo[r];  // ignored rows hold 0
        c += vo[r];
        if (clean) {
            const int64_t g = ind ? ind[r] : r;
            if (g < 0 || g >= n_clean) bad = 1;
            else p += clean[g] ? 1.0f : 0.0f;
        }
    }
    rs[tid] = s;
    rc[tid] = c;
    rp[tid] = p;
    if (bad) atomicOr(err, 1);
    __syncthreads();
    for (int h = 512; h > 0; h >>= 1) {
        if (tid < h) {
            rs[tid] += rs[tid + h];
            rc[tid] += rc[tid + h];
            rp[tid] += rp[tid + h];
        }
        __syncthreads();
    }
    if (tid == 0) {
        out[o] = rs[0] / rc[0];                     // 0/0 = NaN, as torch's empty mean
        out[2 + m] = clean ? rp[0] / static_cast<float>(R) : NAN;
        ws[6 * B + o] = rc[0];
    }
}

// d y_m[r] = g / cnt_m (softmax(y_m[r]) - onehot) for the rows the other
// model selected, 0 elsewhere (rows [0, B) all written)
__global__ __launch_bounds__(256) void k_ct_bwd(const float *__restrict__ y, int64_t ld, int B, int C,
                                                const int64_t *__restrict__ t, int64_t ignore,
                                                const float *__restrict__ ws, int m,
                                                const float *__restrict__ g, float *__restrict__ dy,
                                                int64_t ldd) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= B) return;
    const float *xr = y + static_cast<int64_t>(r) * ld;
    float *dr = dy + static_cast<int64_t>(r) * ldd;
    const int64_t c = t[r];
    if (ws[4 * B + m * B + r] == 0.0f || c == ignore) {
        for (int k = lane; k < C; k += 64) dr[k] = 0.0f;
        return;
    }
    const float lse = row_lse(xr, C, lane);
    const float scale = *g / ws[6 * B + m];
    for (int k = lane; k < C; k += 64) {
        const float p = expf(xr[k] - lse);
        dr[k] = scale * (p - (k == c ? 1.0f : 0.0f));
    }
}

}  // namespace
}  // namespace ngnn

using namespace ngnn;

extern "C" size_t ngnn_seed_xent_workspace_bytes(int64_t B) {
    return B > 0 ? sizeof(float) * 3 * static_cast<size_t>(B) + 256 : 0;
}

extern "C" int ngnn_seed_xent_fwd(const float *logits, int64_t ld, int64_t B, int64_t C,
                                  const int64_t *y, int64_t ignore_index, float *loss, float *count,
                                  void *ws, size_t ws_bytes, void *stream) {
    NGNN_RETURN_IF(!logits || !y || !loss || !count || !ws || B <= 0 || C <= 0, NGNN_E_ARG);
    NGNN_RETURN_IF(ld < C, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(B) || !fits_i32(C), NGNN_E_RANGE);
    NGNN_RETURN_IF(ws_bytes < ngnn_seed_xent_workspace_bytes(B) || !aligned(ws, 16), NGNN_E_WORKSPACE);
    float *w = static_cast<float *>(ws);
    hipLaunchKernelGGL(k_xent_rows, dim3(static_cast<unsigned>(ceil_div(B, 4))), dim3(256), 0,
                       as_stream(stream), logits, ld, (int)B, (int)C, y, ignore_index, w);
    int rc = launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL(k_xent_sum, dim3(1), dim3(256), 0, as_stream(stream), w, (int)B, loss, count);
    return launch_status();
}

extern "C" int ngnn_seed_xent_fwd_grad(const float *logits, int64_t ld, int64_t B, int64_t C,
                                       const int64_t *y, int64_t ignore_index, float *loss,
                                       float *count, float *dlogits, int64_t ldd, void *ws,
                                       size_t ws_bytes, void *stream) {
    NGNN_RETURN_IF(!logits || !y || !loss || !count || !dlogits || !ws || B <= 0 || C <= 0,
                   NGNN_E_ARG);
    NGNN_RETURN_IF(ld < C || ldd < C, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(B) || !fits_i32(C), NGNN_E_RANGE);
    NGNN_RETURN_IF(ws_bytes < ngnn_seed_xent_workspace_bytes(B) || !aligned(ws, 16), NGNN_E_WORKSPACE);
    float *w = static_cast<float *>(ws);
    hipStream_t st = as_stream(stream);
    if (B > kXentFusedMaxB) {
        // large seed sets (a full-batch loader): rows, fixed-order sum, then the
        // gradient rows at unit scale -- O(B) label reads
        const unsigned grid = static_cast<unsigned>(ceil_div(B, 4));
        hipLaunchKernelGGL(k_xent_rows, dim3(grid), dim3(256), 0, st, logits, ld, (int)B, (int)C, y,
                           ignore_index, w);
        hipLaunchKernelGGL(k_xent_sum, dim3(1), dim3(256), 0, st, w, (int)B, loss, count);
        hipLaunchKernelGGL(k_xent_bwd, dim3(grid), dim3(256), 0, st, logits, ld, (int)B, (int)C, y,
                           ignore_index, w, nullptr, count, dlogits, ldd);
        return launch_status();
    }
    // the ticket sits past the row-loss area of ngnn_seed_xent_fwd (3 B floats)
    uint32_t *ticket = reinterpret_cast<uint32_t *>(w + 3 * B);
    hipLaunchKernelGGL(k_xent_fused, dim3(static_cast<unsigned>(ceil_div(B, 4))), dim3(256), 0,
                       as_stream(stream), logits, ld, (int)B, (int)C, y, ignore_index, w, ticket,
                       loss, count, dlogits, ldd);
    return launch_status();
}

extern "C" int ngnn_seed_xent_bwd(const float *logits, int64_t ld, int64_t B, int64_t C,
                                  const int64_t *y, int64_t ignore_index, const void *ws,
                                  const float *grad_scale, const float *count, float *dlogits,
                                  int64_t ldd, void *stream) {
    NGNN_RETURN_IF(!logits || !y || !ws || !grad_scale || !count || !dlogits || B <= 0 || C <= 0,
                   NGNN_E_ARG);
    NGNN_RETURN_IF(ld < C || ldd < C, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(B) || !fits_i32(C), NGNN_E_RANGE);
    hipLaunchKernelGGL(k_xent_bwd, dim3(static_cast<unsigned>(ceil_div(B, 4))), dim3(256), 0,
                       as_stream(stream), logits, ld, (int)B, (int)C, y, ignore_index,
                       static_cast<const float *>(ws), grad_scale, count, dlogits, ldd);
    return launch_status();
}

extern "C" size_t ngnn_ct_loss_workspace_bytes(int64_t B) {
    return B > 0 ? sizeof(float) * (6 * static_cast<size_t>(B) + 2) + sizeof(int) + 256 : 0;
}

extern "C" int ngnn_ct_loss_fwd(const float *y1, int64_t ld1, const float *y2, int64_t ld2, int64_t B,
                                int64_t C, const int64_t *y_noise, int64_t ignore_index,
                                int64_t num_remember, const int64_t *ind, const uint8_t *noise_or_not,
                                int64_t n_noise, float *out, int64_t *ind1_sorted,
                                int64_t *ind2_sorted, void *ws, size_t ws_bytes, int *err,
                                void *stream) {
    NGNN_RETURN_IF(!y1 || !y2 || !y_noise || !out || !ind1_sorted || !ind2_sorted || !ws || !err,
                   NGNN_E_ARG);
    NGNN_RETURN_IF(B <= 0 || C <= 0 || num_remember < 0 || num_remember > B, NGNN_E_ARG);
    NGNN_RETURN_IF(noise_or_not && n_noise <= 0, NGNN_E_ARG);
    NGNN_RETURN_IF(ld1 < C || ld2 < C || B > kCtMaxB, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(C), NGNN_E_RANGE);
    NGNN_RETURN_IF(ws_bytes < ngnn_ct_loss_workspace_bytes(B) || !aligned(ws, 16), NGNN_E_WORKSPACE);
    float *w = static_cast<float *>(ws);
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(k_ct_rows, dim3(static_cast<unsigned>(ceil_div(2 * B, 4))), dim3(256), 0, st,
                       y1, ld1, y2, ld2, (int)B, (int)C, y_noise, ignore_index, w);
    int rc = launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL(k_ct_select, dim3(2), dim3(1024), 0, st, w, (int)B, (int)num_remember, ind,
                       noise_or_not, n_noise, ind1_sorted, ind2_sorted, out, err);
    return launch_status();
}

extern "C" int ngnn_ct_loss_bwd(int model, const float *y, int64_t ld, int64_t B, int64_t C,
                                const int64_t *y_noise, int64_t ignore_index, const void *ws,
                                const float *grad, float *dy, int64_t ldd, void *stream) {
    NGNN_RETURN_IF(model < 0 || model > 1 || !y || !y_noise || !ws || !grad || !dy, NGNN_E_ARG);
    NGNN_RETURN_IF(B <= 0 || C <= 0, NGNN_E_ARG);
    NGNN_RETURN_IF(ld < C || ldd < C || B > kCtMaxB, NGNN_E_SHAPE);
    NGNN_RETURN_IF(!fits_i32(C), NGNN_E_RANGE);
    hipLaunchKernelGGL(k_ct_bwd, dim3(static_cast<unsigned>(ceil_div(B, 4))), dim3(256), 0,
                       as_stream(stream), y, ld, (int)B, (int)C, y_noise, ignore_index,
                       static_cast<const float *>(ws), model, grad, dy, ldd);
    return launch_status();
}
