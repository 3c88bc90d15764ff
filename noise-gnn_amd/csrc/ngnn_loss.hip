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
    const float scale = *g / *count;
    for (int c = lane; c < C; c += 64) {
        const float p = expf(xr[c] - lse);
        dr[c] = scale * (p - (c == t ? 1.0f : 0.0f));
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
