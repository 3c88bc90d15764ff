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

// A operand from LDS (W fragments, 1 KiB per ds_read_b128 per wave, the
// dense kernel's pattern): 4 n-tiles per step, next step's fragments read
// while the current 16 MFMAs issue; B from registers.
__global__ __launch_bounds__(256) void k_mfma_lds(float *out, int iters, float seed) {
    __shared__ v4f w[16 * 64];  // 16 fragments
    for (int i = threadIdx.x; i < 16 * 64; i += 256) w[i] = v4f{seed, seed, seed, seed};
    __syncthreads();
    const int lane = threadIdx.x & 63;
    v4f acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = v4f{0.f, 0.f, 0.f, 0.f};
    v4f b = v4f{seed, seed, seed, seed};
    for (int it = 0; it < iters; ++it) {
        v4f wb[2][4];
#pragma unroll
        for (int h = 0; h < 4; ++h) wb[0][h] = w[h * 64 + lane];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if (s + 1 < 4)
#pragma unroll
                for (int h = 0; h < 4; ++h) wb[(s + 1) & 1][h] = w[((s + 1) * 4 + h) * 64 + lane];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int h = 0; h < 4; ++h)
                    acc[s * 4 + h] = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[s & 1][h][i], b[i], acc[s * 4 + h], 0, 0, 0);
        }
        b[0] += 1e-7f;
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
    for (int per_cu : {1, 2}) {  // LDS-fed A operand; iters/4 outer steps of 64 MFMAs
        const int grid = 256 * per_cu;
        const int it2 = iters / 4;
        hipLaunchKernelGGL(k_mfma_lds, dim3(grid), dim3(256), 0, 0, out, it2, 1.0f);
        (void)hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_mfma_lds, dim3(grid), dim3(256), 0, 0, out, it2, 1.0f);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double flops = 5.0 * grid * 4.0 * it2 * 64 * (16 * 16 * 4 * 2);
        printf("LDS-A wg/CU=%d  %.3f ms  %.1f TFLOP/s\n", per_cu, ms / 5, flops / (ms * 1e-3) / 1e12);
    }
    return 0;
}
