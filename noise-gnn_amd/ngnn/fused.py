"""Whole-stack SAGE forward/backward on the fused kernels.

``SAGE.forward`` (sage.py:30-40) runs, per layer, ``conv -> relu -> dropout``.
Here one autograd node covers the whole stack:

forward, per layer: ``ngnn_sage_fwd`` — gather-aggregate + fp32 MFMA for
``[x | agg] . [W_r; W_l]^T + b`` + ReLU + dropout (hash RNG) in ONE launch;
weights are re-packed into MFMA fragment order each call (~100 KB, they change
every optimiser step).

backward: the loss of every reference pipeline reads only the seed rows
(``out[:batch_size]``, pipeline.py:155), so the output gradient is zero past
row R.  ``ngnn_row_extent`` finds R on the device; each layer's backward then
touches only rows < R (weight / bias gradients, the root-term input gradient)
and the in-edges of those rows (the transposed aggregation), and the input
gradient of the layer below is nonzero only on rows < R' =
max(R, 1 + max source of those edges) (``ngnn_block_prefix_stats``).  On a
NeighborLoader block this is R = batch_size at the top and R' = seeds + hop-1
nodes below it: ~10x less backward work than the dense autograd graph, and
exactly the same result (the skipped rows contribute exact zeros).
One small host read per layer (R, nnz, R') sizes the row-prefix products.
"""
from __future__ import annotations

import torch

from . import _lib, _timing
from .block import Block, build_csr
from .ops import _SegmentAggregate  # noqa: F401  (same kernels, shared checks)

_SAGE_MAX_FO = 512


def pack_weight(w: torch.Tensor) -> torch.Tensor:
    Fo, K = w.shape
    lib = _lib.load()
    nbytes = lib.ngnn_pack_weight_bytes(Fo, K)
    packed = torch.empty(nbytes // 4, dtype=torch.float32, device=w.device)
    w = w.detach()
    if w.stride(1) != 1:
        w = w.contiguous()
    rc = lib.ngnn_pack_weight(_lib.ptr(w), w.stride(0), Fo, K, _lib.ptr(packed),
                              _lib.stream_handle(w.device))
    _lib.check(rc, "ngnn_pack_weight")
    return packed


def sage_layer_fwd(x: torch.Tensor, block: Block, reduce: str, wl, bl, wr, relu: bool,
                   p_drop: float, seed: int) -> torch.Tensor:
    """One fused SAGEConv(+relu+dropout) layer, no autograd."""
    N, K = x.shape
    Fo = wl.shape[0]
    out = torch.empty(N, Fo, dtype=torch.float32, device=x.device)
    pl, pr = pack_weight(wl), pack_weight(wr)
    nbytes = (N * K + block.E * (K + 1) + N * Fo) * 4 + (N + 1) * 4
    with _timing.span("sage_fwd", nbytes):
        rc = _lib.load().ngnn_sage_fwd(
            _lib.ptr(x), x.stride(0), K, N, _lib.ptr(block.rowptr), _lib.ptr(block.col),
            _lib.REDUCE[reduce], _lib.ptr(pl), _lib.ptr(pr), _lib.ptr(bl), Fo, _lib.ptr(out),
            out.stride(0), int(relu), float(p_drop), seed & (2**64 - 1),
            _lib.stream_handle(x.device))
    _lib.check(rc, "ngnn_sage_fwd")
    return out


def _seg_agg(x, rowptr, col, n_dst, reduce):
    F = x.size(1)
    out = torch.empty(n_dst, F, dtype=torch.float32, device=x.device)
    rc = _lib.load().ngnn_seg_agg_fwd(_lib.ptr(x), x.stride(0), F, _lib.ptr(rowptr), _lib.ptr(col),
                                      n_dst, _lib.REDUCE[reduce], _lib.F32, _lib.ptr(out),
                                      out.stride(0), _lib.stream_handle(x.device))
    _lib.check(rc, "ngnn_seg_agg_fwd")
    return out


def _transposed_prefix(block: Block, R: int, nnz: int, n_src_rows: int):
    """Source-grouped CSR of the edges into target rows < R (edge order kept)."""
    rp = block.rowptr
    dev = rp.device
    if nnz == 0:
        return torch.zeros(n_src_rows + 1, dtype=torch.int32, device=dev), None
    deg = (rp[1:R + 1] - rp[:R]).long()
    dst = torch.repeat_interleave(torch.arange(R, device=dev), deg, output_size=nnz)
    src = block.col[:nnz].long()
    t = build_csr(src, dst, n_src_rows, keys_sorted=False)
    return t.rowptr, t.col


def _seg_agg_bwd(g, block, R, rowptr_t, col_t, n_src_rows, reduce, x=None, agg=None):
    """sum_{e into rows < R, src_e = j} d(reduce)/dx_j, rows j < n_src_rows."""
    F = g.size(1)
    lib = _lib.load()
    gx = torch.empty(n_src_rows, F, dtype=torch.float32, device=g.device)
    red = _lib.REDUCE[reduce]
    ws, ws_bytes = None, 0
    if red == _lib.REDUCE["max"]:
        ws_bytes = lib.ngnn_seg_agg_bwd_workspace_bytes(R, F, red)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=g.device)
    E_used = int(col_t.numel()) if col_t is not None else 0
    nbytes = E_used * (F * 4 + 12) + (n_src_rows + 1) * 4 + n_src_rows * F * 4
    with _timing.span("seg_agg_bwd", nbytes):
        rc = lib.ngnn_seg_agg_bwd(
            _lib.ptr(g), g.stride(0), F, _lib.ptr(block.rowptr), _lib.ptr(block.col), R,
            _lib.ptr(rowptr_t), _lib.ptr(col_t), n_src_rows, red, _lib.F32,
            _lib.ptr(x), x.stride(0) if x is not None else F,
            _lib.ptr(agg), agg.stride(0) if agg is not None else F,
            _lib.ptr(gx), gx.stride(0), _lib.ptr(ws), ws_bytes, _lib.stream_handle(g.device))
    _lib.check(rc, "ngnn_seg_agg_bwd")
    return gx


class _SAGEStack(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, block: Block, reduce: str, p_drop: float, seed: int, *params):
        L = len(params) // 3
        acts = [x]
        h = x
        for i in range(L):
            wl, bl, wr = params[3 * i:3 * i + 3]
            last = i == L - 1
            h = sage_layer_fwd(h, block, reduce, wl, bl, wr, relu=not last,
                               p_drop=0.0 if last else p_drop, seed=seed + 7919 * i)
            acts.append(h)
        ctx.block, ctx.reduce, ctx.p_drop, ctx.L = block, reduce, p_drop, L
        ctx.save_for_backward(*acts, *params)
        return h

    @staticmethod
    def backward(ctx, dout):
        block, reduce, p, L = ctx.block, ctx.reduce, ctx.p_drop, ctx.L
        saved = ctx.saved_tensors
        acts, params = saved[:L + 1], saved[L + 1:]
        lib = _lib.load()
        dev = dout.device
        stream = _lib.stream_handle(dev)
        need_dx = ctx.needs_input_grad[0]
        grads = [None] * (3 * L)
        N = block.n_dst
        dy = dout.contiguous()
        # R for the top layer: last nonzero row of the output gradient
        st = torch.zeros(4, dtype=torch.int32, device=dev)
        _lib.check(lib.ngnn_row_extent(_lib.ptr(dy), dy.stride(0), N, dy.size(1), _lib.ptr(st),
                                       stream), "ngnn_row_extent")
        R = None
        dx_full = None
        for i in reversed(range(L)):
            h_in, y = acts[i], acts[i + 1]
            wl, bl, wr = params[3 * i:3 * i + 3]
            need_dh = i > 0 or need_dx
            if R is None or need_dh:
                _lib.check(lib.ngnn_block_prefix_stats(_lib.ptr(block.rowptr), _lib.ptr(block.col),
                                                       -1 if R is None else R, block.E,
                                                       _lib.ptr(st), stream),
                           "ngnn_block_prefix_stats")
                s = st.tolist()  # host read: R, nnz, R'
                R, nnz, R_in = s[0], s[1], max(s[2], s[0])
            else:
                nnz = R_in = None
            K = h_in.size(1)
            if R == 0:
                for j, prm in enumerate((wl, bl, wr)):
                    grads[3 * i + j] = torch.zeros_like(prm)
                dy = torch.zeros(0, K, device=dev)
                R = 0
                continue
            dz = dy[:R]
            if i != L - 1:
                # relu + dropout backward from the stored post-activation: y > 0 <=> kept & pre > 0
                mask = y[:R] > 0
                dz = dz * mask
                if p > 0.0:
                    dz = dz * (1.0 / (1.0 - p))
            dz = dz.contiguous()
            hR = h_in[:R]
            agg = _seg_agg(h_in, block.rowptr, block.col, R, reduce)
            grads[3 * i + 0] = dz.t().mm(agg)          # dW_l
            grads[3 * i + 1] = dz.sum(0)               # db_l
            grads[3 * i + 2] = dz.t().mm(hR)           # dW_r
            if not need_dh:
                continue
            # input gradient: root term on rows < R, transposed aggregation on rows < R_in
            dagg = dz.mm(wl)
            rpt, colt = _transposed_prefix(block, R, nnz, R_in)
            dh = _seg_agg_bwd(dagg, block, R, rpt, colt, R_in, reduce, x=h_in, agg=agg)
            dh[:R].addmm_(dz, wr)
            if i == 0:
                dx_full = torch.zeros(N, K, dtype=dout.dtype, device=dev)
                dx_full[:R_in] = dh
            dy = dh
            R = R_in
            st.zero_()
            st[0] = R
        return (dx_full, None, None, None, None, *grads)


def sage_stack_supported(model, x) -> bool:
    if not x.is_cuda or x.dtype != torch.float32 or x.dim() != 2:
        return False
    if getattr(model, "use_bn", False):
        return False
    aggr = model.convs[0].aggr
    for conv in model.convs:
        if conv.aggr != aggr or conv.out_channels > _SAGE_MAX_FO:
            return False
    return True


def sage_stack(model, x, block: Block, seed: int) -> torch.Tensor:
    params = []
    for conv in model.convs:
        params += [conv.lin_l.weight, conv.lin_l.bias, conv.lin_r.weight]
    p = model.dropout if model.training else 0.0
    aggr = "sum" if model.convs[0].aggr == "add" else model.convs[0].aggr
    xc = x if (x.stride(1) == 1 and x.stride(0) >= x.size(1)) else x.contiguous()
    return _SAGEStack.apply(xc, block, aggr, float(p), int(seed), *params)
