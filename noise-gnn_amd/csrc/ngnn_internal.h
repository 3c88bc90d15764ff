// Internal helpers shared by the ngnn HIP translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "ngnn.h"

#define NGNN_RETURN_IF(cond, code) \
    do {                           \
        if (cond) return (code);   \
    } while (0)

namespace ngnn {

constexpr int kWave = 64;  // CDNA wavefront

inline int launch_status() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? NGNN_OK : static_cast<int>(e);
}

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

inline bool fits_i32(int64_t v) { return v >= 0 && v <= INT32_MAX; }

inline bool aligned(const void *p, size_t a) {
    return (reinterpret_cast<uintptr_t>(p) % a) == 0;
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

int num_cus();  // compute units of the current device (cached; ngnn_sage_rt.hip)

// The graph slot's contract gate (ABI 20): the slot kernel keeps, in a
// 64-bit word, (gen << 32 | bad bits) of the last load that broke the
// block's contract (atomicMax: the newest generation wins); gen_word is the
// slot's r_next word, whose high half is the current load's generation.  A
// step whose block broke the contract leaves the parameters and the step
// count untouched.  gate NULL: never gated.
__device__ __forceinline__ bool slot_gated(const uint64_t *gate, const int64_t *gen_word) {
    if (!gate || !gen_word) return false;
    const uint64_t g = *gate;
    return (g & 0xffffffffull) != 0 && (g >> 32) == (static_cast<uint64_t>(*gen_word) >> 32);
}

}  // namespace ngnn
