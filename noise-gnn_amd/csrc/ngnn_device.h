// Device helpers shared by the fused SAGE kernels (forward and backward).
#pragma once

#include "ngnn_internal.h"

namespace ngnn {

typedef float v4f __attribute__((ext_vector_type(4)));

// Tile geometry of the fused layer kernels: a 256-thread workgroup owns 64
// target rows; K is staged through ONE LDS buffer in 128-column chunks.
constexpr int kBM = 64;
constexpr int kKC = 128;
constexpr int kLDA = kKC + 4;  // padded row stride (floats): 528 B
constexpr int kTileFloats = kBM * kLDA;

// torch amax semantics: NaN propagates, otherwise the larger value wins.
__device__ __forceinline__ float nanmax(float acc, float v) {
    return (acc != acc) ? acc : ((v != v || v > acc) ? v : acc);
}

// ---- dropout RNG: counter-based, keyed by (seed, row, col); the keep mask is
// never stored.  keep <=> (hash >> 8) >= thresh, thresh = ceil(p * 2^24).
// Host replica: tests/test_gpu_fused.py::dropout_keep.
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

struct Dropout {
    uint32_t s0, s1, thresh;  // thresh == 0: no dropout; > 2^24: drop all
    float scale;
    __device__ __forceinline__ uint32_t row_key(uint32_t row) const { return lowbias32(row ^ s0); }
    __device__ __forceinline__ bool keep(uint32_t rkey, uint32_t col) const {
        return (lowbias32(lowbias32(rkey + col) ^ s1) >> 8) >= thresh;
    }
};

inline Dropout make_dropout(float p, uint64_t seed) {
    Dropout d;
    d.s0 = static_cast<uint32_t>(seed);
    d.s1 = static_cast<uint32_t>(seed >> 32);
    if (!(p > 0.0f)) {
        d.thresh = 0;
        d.scale = 1.0f;
    } else if (p >= 1.0f) {
        d.thresh = (1u << 24) + 1;  // nothing kept
        d.scale = 0.0f;
    } else {
        const double t = static_cast<double>(p) * 16777216.0;
        uint32_t ti = static_cast<uint32_t>(t);
        if (static_cast<double>(ti) < t) ++ti;  // ceil
        d.thresh = ti;
        d.scale = 1.0f / (1.0f - p);
    }
    return d;
}

}  // namespace ngnn
