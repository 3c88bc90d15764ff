/*
 * seg_agg.c — plain-C restatement of the per-destination aggregation that
 * PyTorch Geometric 2.5.1 performs inside SAGEConv / GCNConv for a Tensor
 * edge_index.  ORACLE / TEST INFRASTRUCTURE ONLY: never linked into the product.
 *
 * Reference call sites: src/models/layers/sage.py:34 (conv(x, edge_index)),
 * src/models/layers/convolution.py:31; arithmetic in PyG 2.5.1 [ext]
 * (docs/requirements.txt:11) — MessagePassing.propagate + utils.scatter:
 *   x_j   = x.index_select(0, edge_index[0])
 *   sum : zeros(N,F).scatter_add_(0, dst, x_j)                 (edge order)
 *   mean: sum / zeros(N).scatter_add_(0, dst, 1).clamp(min=1)
 *   max : zeros(N,F).scatter_reduce_(0, dst, x_j, 'amax', include_self=False)
 * Backward restates torch autograd of those ops (index_select -> index_add_
 * in edge order; scatter_reduce amax -> even split over ties, where the
 * zero-initialised `self` counts as a tie when the maximum equals 0:
 * torch/csrc/autograd/FunctionsManual.cpp scatter_reduce_backward [ext]).
 *
 * All loops run in edge order so fp32 results are bit-comparable with the
 * sequential CPU ATen kernels.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { RED_SUM = 0, RED_MEAN = 1, RED_MAX = 2 };

static float nanmax_first(float acc, float v) {
    /* torch amax propagates NaN */
    if (isnan(acc)) return acc;
    if (isnan(v)) return v;
    return v > acc ? v : acc;
}

int oracle_agg_fwd(const float *x, int64_t ldx, int64_t F, const int64_t *src,
                   const int64_t *dst, int64_t E, int64_t n_dst, int reduce,
                   float *out, int64_t ldo) {
    float *cnt = (float *)calloc((size_t)(n_dst > 0 ? n_dst : 1), sizeof(float));
    if (!cnt) return -1;
    for (int64_t i = 0; i < n_dst; ++i) memset(out + i * ldo, 0, sizeof(float) * (size_t)F);
    for (int64_t e = 0; e < E; ++e) {
        const int64_t s = src[e], d = dst[e];
        const float *xr = x + s * ldx;
        float *o = out + d * ldo;
        if (reduce == RED_MAX) {
            if (cnt[d] == 0.0f) {
                for (int64_t f = 0; f < F; ++f) o[f] = xr[f];
            } else {
                for (int64_t f = 0; f < F; ++f) o[f] = nanmax_first(o[f], xr[f]);
            }
        } else {
            for (int64_t f = 0; f < F; ++f) o[f] += xr[f];
        }
        cnt[d] += 1.0f;
    }
    if (reduce == RED_MEAN) {
        for (int64_t i = 0; i < n_dst; ++i) {
            const float c = cnt[i] < 1.0f ? 1.0f : cnt[i];
            for (int64_t f = 0; f < F; ++f) out[i * ldo + f] = out[i * ldo + f] / c;
        }
    }
    free(cnt);
    return 0;
}

/* grad_x[n_src, F] = d(agg)/dx applied to grad_out[n_dst, F].
 * For max, `agg` is the forward output and `x` the forward input. */
int oracle_agg_bwd(const float *grad_out, int64_t ldg, int64_t F, const int64_t *src,
                   const int64_t *dst, int64_t E, int64_t n_src, int64_t n_dst,
                   int reduce, const float *x, int64_t ldx, const float *agg,
                   int64_t lda, float *grad_x, int64_t ldgx) {
    for (int64_t j = 0; j < n_src; ++j) memset(grad_x + j * ldgx, 0, sizeof(float) * (size_t)F);
    if (reduce == RED_SUM || reduce == RED_MEAN) {
        float *cnt = (float *)calloc((size_t)(n_dst > 0 ? n_dst : 1), sizeof(float));
        if (!cnt) return -1;
        for (int64_t e = 0; e < E; ++e) cnt[dst[e]] += 1.0f;
        for (int64_t e = 0; e < E; ++e) {
            const int64_t s = src[e], d = dst[e];
            const float c = cnt[d] < 1.0f ? 1.0f : cnt[d];
            for (int64_t f = 0; f < F; ++f) {
                const float g = grad_out[d * ldg + f];
                grad_x[s * ldgx + f] += (reduce == RED_MEAN) ? g / c : g;
            }
        }
        free(cnt);
        return 0;
    }
    /* max: N[d,f] = [agg==0] + #{e into d : x[src_e,f] == agg[d,f]} */
    float *ties = (float *)calloc((size_t)(n_dst > 0 ? n_dst : 1) * (size_t)(F > 0 ? F : 1), sizeof(float));
    if (!ties) return -1;
    for (int64_t i = 0; i < n_dst; ++i)
        for (int64_t f = 0; f < F; ++f) ties[i * F + f] = (agg[i * lda + f] == 0.0f) ? 1.0f : 0.0f;
    for (int64_t e = 0; e < E; ++e) {
        const int64_t s = src[e], d = dst[e];
        for (int64_t f = 0; f < F; ++f)
            if (x[s * ldx + f] == agg[d * lda + f]) ties[d * F + f] += 1.0f;
    }
    for (int64_t e = 0; e < E; ++e) {
        const int64_t s = src[e], d = dst[e];
        for (int64_t f = 0; f < F; ++f) {
            const float gd = grad_out[d * ldg + f] / ties[d * F + f];
            const float m = (x[s * ldx + f] == agg[d * lda + f]) ? 1.0f : 0.0f;
            grad_x[s * ldgx + f] += m * gd;
        }
    }
    free(ties);
    return 0;
}
