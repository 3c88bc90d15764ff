// Standalone calibration: achievable v_mfma_f32_16x16x4_f32 rate on this box
// (register operands only, 16 independent accumulators per wave, like the
// fused layer kernel's 4x4 tile), at 1..4 workgroups of 256 threads per CU.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_peak.hip -o /tmp/mfma_peak && /tmp/mfma_peak
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_mfma(float *out, int iters, float seed) {
    v4f acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = v4f{0.f, 0.f, 0.f, 0.f};
    float a = seed + threadIdx.x * 1e-3f, b = seed - threadIdx.x * 1e-3f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
        a += 1e-7f;
    }
    float s = 0.f;
    for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
    float *out;
    (void)hipMalloc(&out, sizeof(float) * 256 * 4096);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 2000;
    for (int per_cu : {1, 2, 3, 4}) {
        const int grid = 256 * per_cu;
        hipLaunchKernelGGL(k_mfma, dim3(grid), dim3(256), 0, 0, out, iters, 1.0f);
        (void)hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_mfma, dim3(grid), dim3(256), 0, 0, out, iters, 1.0f);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double flops = 5.0 * grid * 4.0 /*waves*/ * iters * 16 * (16 * 16 * 4 * 2);
        printf("wg/CU=%d  %.3f ms  %.1f TFLOP/s\n", per_cu, ms / 5, flops / (ms * 1e-3) / 1e12);
    }
    return 0;
}
