// Device helpers shared by the fused SAGE kernels (forward and backward).
#pragma once

#include "ngnn_internal.h"

namespace ngnn {

// a load through a global (address-space 1) pointer: a pointer read from
// memory (e.g. a graph slot's device word) is otherwise generic and becomes a
// flat load, which also counts against lgkmcnt and serialises LDS waits
template <typename T>
__device__ __forceinline__ T gload(const T *p, int64_t i) {
    return ((const __attribute__((address_space(1))) T *)(p))[i];
}

typedef float v4f __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));

// ---- raw buffer access (LLVM intrinsics by name).  A resource covers
// [base, base + bytes) (word3 = 0x00020000: raw, 32-bit element format for
// gfx950); loads past the range return 0 and stores past it are dropped, so
// row/column bounds become one per-lane offset select instead of branches.
__device__ v4f buf_load4(i32x4 rsrc, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4f32");
__device__ float buf_load1(i32x4 rsrc, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.f32");
__device__ int buf_load1i(i32x4 rsrc, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.i32");
__device__ i32x2 buf_load2i(i32x4 rsrc, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.v2i32");
__device__ i32x4 buf_load4i(i32x4 rsrc, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4i32");
__device__ void buf_store4(v4f v, i32x4 rsrc, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.store.v4f32");
__device__ void buf_store1(float v, i32x4 rsrc, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.store.f32");
__device__ void buf_store2i(i32x2 v, i32x4 rsrc, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.store.v2i32");

__device__ __forceinline__ i32x4 make_rsrc(const void *p, uint32_t bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    i32x4 r;
    r.x = static_cast<int>(static_cast<uint32_t>(a));
    r.y = static_cast<int>(static_cast<uint32_t>(a >> 32));
    r.z = static_cast<int>(bytes);
    r.w = 0x00020000;
    return r;
}
// The same for a resource the compiler cannot prove wave-uniform (derived
// from a loaded value: a graph slot's x address, a device row count) but that
// is: readfirstlane puts it in SGPRs, else every buffer access is wrapped in a
// waterfall loop behind an s_waitcnt vmcnt(0) that drains the prefetches.
__device__ __forceinline__ i32x4 make_rsrc_u(const void *p, uint32_t bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    i32x4 r;
    r.x = __builtin_amdgcn_readfirstlane(static_cast<int>(static_cast<uint32_t>(a)));
    r.y = __builtin_amdgcn_readfirstlane(static_cast<int>(static_cast<uint32_t>(a >> 32)));
    r.z = __builtin_amdgcn_readfirstlane(static_cast<int>(bytes));
    r.w = 0x00020000;
    return r;
}
// 4 bf16 (two little-endian words: element 2j in the low half of word j) ->
// 4 floats, exactly
__device__ __forceinline__ v4f bf16x4_to_f32(i32x2 w) {
    v4f o;
    o[0] = __int_as_float(w.x << 16);
    o[1] = __int_as_float(w.x & static_cast<int>(0xffff0000u));
    o[2] = __int_as_float(w.y << 16);
    o[3] = __int_as_float(w.y & static_cast<int>(0xffff0000u));
    return o;
}

// ---- H2 scaling (two-layer forward and backward): powers of two that put a
// block's max |v| in [2^14, 2^15) before an fp16 split, and the cross-lane
// maxima that find it
// e with max|v| 2^e in [2^14, 2^15) (0 -> 15; inf / NaN rows stay inf / NaN)
__device__ __forceinline__ int h2_exp(float amax) { return 15 - __builtin_amdgcn_frexp_expf(amax); }

__device__ __forceinline__ v4f ldexp4(v4f v, int e) {
    v4f o;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = __builtin_amdgcn_ldexpf(v[i], e);
    return o;
}

__device__ __forceinline__ float amax4(v4f v) {
    return fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
}

// cross-lane max of non-negative floats (their bit patterns order as ints),
// on VALU only (no LDS round trip): DPP inside a 16-lane row, the gfx950
// permlane swaps across rows
__device__ __forceinline__ float max_xor16(float v) {  // lanes l and l ^ 16
    const int x = __float_as_int(v);
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return __int_as_float(max(static_cast<int>(r[0]), static_cast<int>(r[1])));
}
__device__ __forceinline__ float max_xor32(float v) {  // lanes l and l ^ 32
    const int x = __float_as_int(v);
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return __int_as_float(max(static_cast<int>(r[0]), static_cast<int>(r[1])));
}
__device__ __forceinline__ float max_row16(float v) {  // all 16 lanes of the row
    int x = __float_as_int(v);
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false));  // row_half_mirror
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, false));  // row_mirror
    return __int_as_float(x);
}

// max of a non-negative float over the wave
__device__ __forceinline__ float wave_max(float v) { return max_xor32(max_xor16(max_row16(v))); }

// The training step's seed-row cross entropy computed by the narrow output
// launch (include/ngnn.h ngnn_xent_head; ngnn_sage_rt.hip k_narrow_agg)
struct NarrowHead {
    const int64_t *y;
    int B;
    int64_t ignore;
    float *loss, *count;
    float *dy;
    int64_t ldd;
    float *g;  // nullable: no scatter
    int ldg;
    float *part;       // per-workgroup loss partials
    uint32_t *ticket;  // zero between calls
    const float *cnt_in;  // the valid-label count, written by an earlier launch (nullable: count here)
    int dbg;              // (profiling builds only: time-attribution variants; 0)
    // seed-edge counts per source (nullable): arrays [2][scnt_stride], the
    // word scnt_base[2 scnt_stride] selects this call's; the loss's last
    // adder flips it for the next call (ngnn.h ngnn_xent_head src_count)
    int32_t *scnt_base;
    int scnt_stride;
};

// byte offset that is always outside a resource of < 2 GiB
constexpr int kBufOOB = 0x7fffffff;

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
// never stored.  p is resolved to thresh / 256, thresh = ceil(p * 256) (exact
// for 0, 0.25, 0.5, 0.75, 1); survivors scale by 1 / (1 - thresh / 256), so
// E[out] = in exactly.
//  * byte mode (thresh != 128): one 32-bit hash per column QUAD (4c .. 4c+3),
//    byte j of it decides column 4c + j: keep <=> byte >= thresh;
//  * bit mode (thresh == 128, p = 0.5 -- every config's dropout): one BIT per
//    element, column c of a row is bit c & 31 of the hash of word c >> 5,
//    keep <=> bit set (a hash per 32 columns instead of per 4).
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
    uint32_t s0, s1, thresh;  // thresh == 0: no dropout; 256: drop all
    float scale;
    // one hash per row (seed-mixed), one per column quad: rkey + col/4 are
    // distinct within a row and lowbias32 is a bijection
    __device__ __forceinline__ uint32_t row_key(uint32_t row) const {
        return lowbias32(row ^ s0) ^ s1;
    }
    __device__ __forceinline__ uint32_t quad_hash(uint32_t rkey, uint32_t col) const {
        return lowbias32(rkey + (col >> 2));
    }
    __device__ __forceinline__ bool keep_byte(uint32_t h, uint32_t col) const {
        return ((h >> (8 * (col & 3u))) & 0xffu) >= thresh;
    }
    __device__ __forceinline__ bool bit_mode() const { return thresh == 128u; }
    // bit mode: the hash word of column col and its bit
    __device__ __forceinline__ static uint32_t bit_word(uint32_t col) { return col >> 5; }
    __device__ __forceinline__ static uint32_t bit_index(uint32_t col) { return col & 31u; }
    __device__ __forceinline__ bool keep(uint32_t rkey, uint32_t col) const {
        if (bit_mode()) return (lowbias32(rkey + bit_word(col)) >> bit_index(col)) & 1u;
        return keep_byte(quad_hash(rkey, col), col);
    }
    // the four keep decisions of column quad c4 (columns 4 c4 .. 4 c4 + 3), bit j
    __device__ __forceinline__ uint32_t keep4(uint32_t rkey, uint32_t c4) const {
        if (bit_mode())
            return (lowbias32(rkey + bit_word(4u * c4)) >> bit_index(4u * c4)) & 0xfu;
        const uint32_t h = lowbias32(rkey + c4);
        uint32_t k = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) k |= (((h >> (8 * j)) & 0xffu) >= thresh ? 1u : 0u) << j;
        return k;
    }
    __device__ __forceinline__ void reseed(uint64_t d) {
        s0 ^= static_cast<uint32_t>(d);
        s1 ^= static_cast<uint32_t>(d >> 32);
    }
};

// Layer epilogue: bias, optional ReLU, optional dropout; col_base = global
// column of the launch's column 0 (the dropout key is the global column).
struct Epi {
    const float *bias;
    int relu;
    Dropout drop;
    int col_base;
};

inline Dropout make_dropout(float p, uint64_t seed) {
    Dropout d;
    d.s0 = static_cast<uint32_t>(seed);
    d.s1 = static_cast<uint32_t>(seed >> 32);
    if (!(p > 0.0f)) {
        d.thresh = 0;
        d.scale = 1.0f;
        return d;
    }
    const double t = static_cast<double>(p) * 256.0;
    uint32_t ti = static_cast<uint32_t>(t < 256.0 ? t : 256.0);
    if (static_cast<double>(ti) < t && ti < 256) ++ti;  // ceil
    if (ti == 0) ti = 1;  // p > 0 drops something
    d.thresh = ti;
    d.scale = ti >= 256 ? 0.0f : 256.0f / static_cast<float>(256 - ti);
    return d;
}

// Row-tile forward (ngnn_sage_rt.hip): returns 1 (launch status in *rc) when
// it takes the call, 0 when the shape is outside its envelope.  exact: root
// term on fp32 MFMA (else the 3 x bf16 split when the weights are raw rows).
int sage_fwd_rowtile(const float *x, int64_t ldx, int64_t K, int64_t n_rows,
                     const int32_t *n_rows_dev, const int32_t *rowptr, const int32_t *col,
                     int reduce, const void *wl_packed, const void *wr_packed, const float *bias,
                     int64_t Fo, float *out, int64_t ldo, int relu, float p_drop, uint64_t seed,
                     const uint64_t *seed_dev, float *agg_out, int64_t ld_agg, hipStream_t st,
                     int *rc, int64_t ldw = 0, void *wl_ws = nullptr, size_t wl_ws_bytes = 0,
                     const float *const *x_dev = nullptr, bool exact = true,
                     float *z = nullptr, int64_t ldz = 0, const int64_t *xrow = nullptr,
                     const int64_t *const *xrow_dev = nullptr, int64_t x_rows = 0,
                     const int32_t *col_x = nullptr, bool x_bf16 = false,
                     bool w_bf16 = false, bool wl_prepacked = false, bool agg_pre = false,
                     bool out_bf16 = false, int64_t n_edge_rows = -1,
                     const int32_t *n_edge_rows_dev = nullptr, void *img_ws = nullptr);
// the tail of ngnn_sage_fwd_raw's workspace that holds a slice's prebuilt
// X3 root image (ngnn_root.hip: k_x3_image)
constexpr size_t kImgWsBytes = 160 * 1024;

// Wide-layer forward (ngnn_wide.hip): an aggregate launch into agg_out (or
// the workspace) + a 2-D tiled fp32-MFMA dual GEMM.  Raw [F_out, K] weights.
bool sage_wide_preferred(int64_t K, int64_t Fo, bool exact);
size_t sage_wide_workspace_bytes(int64_t K, int64_t n_rows);
size_t wide_wimg_bytes(int64_t K, int64_t Fo);  // the split-bf16 weight image (at the workspace's tail)
int sage_wide_aggregate(const float *x, int64_t ldx, int64_t K, int64_t n_rows,
                        const int32_t *n_rows_dev, int64_t n_edge_rows,
                        const int32_t *n_edge_rows_dev, const int32_t *rowptr, const int32_t *col,
                        int reduce, float *agg, int64_t ld_agg, hipStream_t st,
                        const float *const *x_dev = nullptr);
int sage_fwd_wide(const float *x, int64_t ldx, int64_t K, int64_t n_rows,
                  const int32_t *n_rows_dev, int64_t n_edge_rows, const int32_t *n_edge_rows_dev,
                  const int32_t *rowptr, const int32_t *col, int reduce, const float *wl,
                  const float *wr, int64_t ldw, const float *bias, int64_t Fo, float *out,
                  int64_t ldo, int relu, float p_drop, uint64_t seed, const uint64_t *seed_dev,
                  float *agg_out, int64_t ld_agg, void *ws, size_t ws_bytes, hipStream_t st,
                  bool exact = false, const float *const *x_dev = nullptr);

}  // namespace ngnn
