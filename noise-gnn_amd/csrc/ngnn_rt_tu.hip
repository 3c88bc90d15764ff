// One (NTW, RED) slice of the row-tile kernel's instantiations: the Makefile
// compiles this file once per pair (-DNGNN_RT_TU_NTW=.. -DNGNN_RT_TU_RED=..),
// so the ~300 k_sage_rt variants build in parallel instead of in one unit.
#include "ngnn_sage_rt_kern.h"

#if !defined(NGNN_RT_TU_NTW) || !defined(NGNN_RT_TU_RED)
#error "build with -DNGNN_RT_TU_NTW=<2|3|4|6|8|16> -DNGNN_RT_TU_RED=<0|1|2>"
#endif

namespace ngnn {
#define NGNN_RT_DEFINE(N, R)                                                                  \
    int NGNN_RT_FN(N, R)(const RtArgs &a, bool wl_lds, bool x3, int n_tiles, size_t lds,     \
                         hipStream_t st) {                                                    \
        return dispatch_rt_red<N, R>(a, wl_lds, x3, n_tiles, lds, st);                         \
    }
#define NGNN_RT_DEFINE2(N, R) NGNN_RT_DEFINE(N, R)
NGNN_RT_DEFINE2(NGNN_RT_TU_NTW, NGNN_RT_TU_RED)
}  // namespace ngnn
