// The eager drop-in's two-layer SAGE stack as a C++ autograd node (round 6).
//
// What a user of the reference loop gets after the INTEGRATION.md Option-B
// swap, with no graph capture (pipeline.py:152-169: out = model(x,
// edge_index)[:bs]; F.cross_entropy; loss.backward(); optimizer.step()), runs
// host-bound: the Python autograd Function of ngnn.fused (_SAGEStack) spent
// ~45 us per forward and ~80 us per backward of host time building the C ABI
// calls.  This node makes the same calls -- ngnn_sage2_fwd; ngnn_row_extent,
// ngnn_block_prefix_stats and ngnn_sage2_bwd -- from C++: the same kernels,
// the same arguments as ngnn.fused.sage2_forward / sage2_backward take on that
// path (plain rows, no graph slot, no loss head, every row of h kept), so the
// results are those of the Python node bit for bit.
//
// The library's entry points come in as addresses from the already loaded
// libngnn.so (ngnn._lib), so this module links torch only.  Built in-tree by
// __graft_entry__.build() (torch.utils.cpp_extension); ngnn.fused uses it when
// it loaded and the call qualifies, else its Python node.
#include <torch/extension.h>

#include "ngnn.h"

namespace {

decltype(&ngnn_sage2_fwd) p_fwd = nullptr;
decltype(&ngnn_sage2_bwd) p_bwd = nullptr;
decltype(&ngnn_row_extent) p_rowext = nullptr;
decltype(&ngnn_block_prefix_stats) p_prefix = nullptr;
decltype(&ngnn_strerror) p_strerror = nullptr;

void check(int rc, const char *what) {
    TORCH_CHECK(rc == 0, "ngnn: ", what, ": ", p_strerror ? p_strerror(rc) : "error", " (rc=", rc, ")");
}

void init(int64_t fwd, int64_t bwd, int64_t rowext, int64_t prefix, int64_t strerr) {
    p_fwd = reinterpret_cast<decltype(p_fwd)>(fwd);
    p_bwd = reinterpret_cast<decltype(p_bwd)>(bwd);
    p_rowext = reinterpret_cast<decltype(p_rowext)>(rowext);
    p_prefix = reinterpret_cast<decltype(p_prefix)>(prefix);
    p_strerror = reinterpret_cast<decltype(p_strerror)>(strerr);
}

using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

float *fp(const torch::Tensor &t) { return t.data_ptr<float>(); }

struct Sage2Stack : public torch::autograd::Function<Sage2Stack> {
    // x [N, K0] fp32 rows; the six weights of SAGEConv(K0, H) + SAGEConv(H,
    // F1); the block's target-grouped CSR (int32) and its leading rows with
    // in-edges (n_edge), E edges; yscale: the dropout survivor scale the
    // backward applies (ngnn.fused.dropout_scale); ws_fwd / ws_bwd: the
    // caller's cached workspaces (the backward's zero-filled)
    static torch::Tensor forward(AutogradContext *ctx, const torch::Tensor &x, const torch::Tensor &wl0,
                                 const torch::Tensor &bl0, const torch::Tensor &wr0, const torch::Tensor &wl1,
                                 const torch::Tensor &bl1, const torch::Tensor &wr1, const torch::Tensor &rowptr,
                                 const torch::Tensor &col, int64_t n_edge, int64_t E, int64_t reduce, double p_drop,
                                 double yscale, int64_t seed, const torch::Tensor &ws_fwd,
                                 const torch::Tensor &ws_bwd, int64_t stream) {
        const int64_t N = x.size(0), K0 = x.size(1), H = wl0.size(0), F1 = wl1.size(0);
        const auto opt = x.options();
        auto h = torch::empty({N, H}, opt);
        auto out = torch::empty({N, F1}, opt);
        auto agg0 = torch::empty({N, K0}, opt);
        void *st = reinterpret_cast<void *>(stream);
        check(p_fwd(fp(x), nullptr, nullptr, nullptr, 0, x.stride(0), K0, N, nullptr, n_edge, nullptr,
                    rowptr.data_ptr<int32_t>(), col.data_ptr<int32_t>(), nullptr, static_cast<int>(reduce), fp(wl0),
                    fp(bl0), fp(wr0), wl0.stride(0), H, fp(wl1), fp(bl1), fp(wr1), wl1.stride(0), F1,
                    static_cast<float>(p_drop), static_cast<uint64_t>(seed), nullptr, fp(h), h.stride(0), N, nullptr,
                    fp(agg0), agg0.stride(0), fp(out), out.stride(0), nullptr, NGNN_SAGE2_ALL, ws_fwd.data_ptr(),
                    static_cast<size_t>(ws_fwd.numel()), st),
              "ngnn_sage2_fwd");
        ctx->save_for_backward({x, h, agg0, wl0, bl0, wr0, wl1, bl1, wr1, rowptr, col, ws_bwd});
        ctx->saved_data["E"] = E;
        ctx->saved_data["reduce"] = reduce;
        ctx->saved_data["yscale"] = yscale;
        ctx->saved_data["stream"] = stream;
        return out;
    }

    // every weight gradient from dy (rows of dy that can be nonzero: its row
    // extent; the sources' bound: the block's prefix stats) -- the eager
    // branch of ngnn.fused._SAGEStack.backward
    static variable_list backward(AutogradContext *ctx, variable_list grads) {
        const auto s = ctx->get_saved_variables();
        const auto &x = s[0], &h = s[1], &agg0 = s[2], &wl1 = s[6], &wr1 = s[8], &rowptr = s[9], &col = s[10],
                   &ws = s[11];
        const int64_t E = ctx->saved_data["E"].toInt(), reduce = ctx->saved_data["reduce"].toInt();
        const double yscale = ctx->saved_data["yscale"].toDouble();
        void *st = reinterpret_cast<void *>(ctx->saved_data["stream"].toInt());
        auto dy = grads[0];
        if (dy.stride(1) != 1) dy = dy.contiguous();
        const int64_t N = x.size(0), K0 = x.size(1), F1 = wl1.size(0);
        // bnd[2]: rows of dy that can be nonzero; bnd[1]: their sources' bound
        auto bnd = torch::zeros({3}, rowptr.options());
        int32_t *b = bnd.data_ptr<int32_t>();
        check(p_rowext(fp(dy), dy.stride(0), N, F1, b + 2, st), "ngnn_row_extent");
        check(p_prefix(rowptr.data_ptr<int32_t>(), col.data_ptr<int32_t>(), b + 2, nullptr, b + 1, E, st),
              "ngnn_block_prefix_stats");
        variable_list g(18);
        for (int k = 0; k < 6; ++k) g[1 + k] = torch::empty_like(s[3 + k]);
        check(p_bwd(fp(dy), dy.stride(0), F1, fp(wl1), fp(wr1), wl1.stride(0), fp(h), h.stride(0),
                    static_cast<float>(yscale), fp(x), nullptr, nullptr, nullptr, 0, x.stride(0), K0, fp(agg0),
                    agg0.stride(0), rowptr.data_ptr<int32_t>(), col.data_ptr<int32_t>(), N, b + 2, b + 1,
                    static_cast<int>(reduce), fp(g[4]), fp(g[5]), fp(g[6]), fp(g[1]), fp(g[2]), fp(g[3]), nullptr,
                    nullptr, ws.data_ptr(), static_cast<size_t>(ws.numel()), st),
              "ngnn_sage2_bwd");
        return g;
    }
};

torch::Tensor sage2(const torch::Tensor &x, const torch::Tensor &wl0, const torch::Tensor &bl0,
                    const torch::Tensor &wr0, const torch::Tensor &wl1, const torch::Tensor &bl1,
                    const torch::Tensor &wr1, const torch::Tensor &rowptr, const torch::Tensor &col, int64_t n_edge,
                    int64_t E, int64_t reduce, double p_drop, double yscale, int64_t seed,
                    const torch::Tensor &ws_fwd, const torch::Tensor &ws_bwd, int64_t stream) {
    TORCH_CHECK(p_fwd && p_bwd && p_rowext && p_prefix, "ngnn_eager: init() first");
    return Sage2Stack::apply(x, wl0, bl0, wr0, wl1, bl1, wr1, rowptr, col, n_edge, E, reduce, p_drop, yscale, seed,
                             ws_fwd, ws_bwd, stream);
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
    m.def("init", &init, "the libngnn entry points (addresses)");
    m.def("sage2", &sage2, "the two-layer SAGE stack as one autograd node (eager)");
}
