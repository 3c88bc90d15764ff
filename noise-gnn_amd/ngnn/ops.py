"""Autograd ops over libngnn (no CPU fallback).

``segment_aggregate(x, block, reduce)`` is the drop-in for PyG 2.5.1's
``MessagePassing.propagate`` with ``message = x_j`` and ``aggr`` in
{'mean', 'sum'/'add', 'max'} over a ``Tensor`` edge_index [ext] — the call the
reference makes inside every conv (``sage.py:34``, ``convolution.py:31``).

Forward: ``ngnn_seg_agg_fwd`` over the target-grouped CSR.
Backward: ``ngnn_seg_agg_bwd`` over the source-grouped CSR (a gather, no
atomics), reproducing torch autograd of ``index_select`` + ``scatter_add_``
(and of ``scatter_reduce_(amax)``: even split over ties, the zero ``self``
counting as a tie when the maximum is 0).
"""
from __future__ import annotations

import torch

from . import _lib, _timing
from .block import Block


def _check_features(x: torch.Tensor, name: str = "x") -> torch.Tensor:
    if not x.is_cuda:
        raise RuntimeError(f"ngnn runs on the GPU only: {name} is on the CPU")
    if x.dim() != 2:
        raise ValueError(f"{name} must be 2-D [N, F], got shape {tuple(x.shape)}")
    if x.dtype != torch.float32:
        raise TypeError(f"{name}: only float32 is supported on this path, got {x.dtype}")
    if x.stride(1) != 1 or x.stride(0) < x.size(1):
        x = x.contiguous()
    return x


class _SegmentAggregate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, block: Block, reduce: str):
        x = _check_features(x)
        if x.size(0) != block.n_src:
            raise ValueError(f"x has {x.size(0)} rows but the block has {block.n_src} nodes")
        F = x.size(1)
        out = torch.empty(block.n_dst, F, dtype=x.dtype, device=x.device)
        red = _lib.REDUCE[reduce]
        # algorithmic bytes: gathered rows + col + rowptr + output rows
        nbytes = block.E * (F * 4 + 4) + (block.n_dst + 1) * 4 + block.n_dst * F * 4
        with _timing.span("seg_agg_fwd", nbytes):
            rc = _lib.load().ngnn_seg_agg_fwd(
                _lib.ptr(x), x.stride(0), F, _lib.ptr(block.rowptr), _lib.ptr(block.col),
                block.n_dst, red, _lib.F32, _lib.ptr(out), out.stride(0),
                _lib.stream_handle(x.device))
        _lib.check(rc, "ngnn_seg_agg_fwd")
        ctx.block, ctx.red = block, red
        if red == _lib.REDUCE["max"]:
            ctx.save_for_backward(x, out)
        return out

    @staticmethod
    def backward(ctx, g):
        if not ctx.needs_input_grad[0]:
            return None, None, None
        block, red = ctx.block, ctx.red
        g = _check_features(g, "grad")
        F = g.size(1)
        t = block.transposed()
        gx = torch.empty(block.n_src, F, dtype=g.dtype, device=g.device)
        lib = _lib.load()
        x = agg = ws = None
        ws_bytes = 0
        if red == _lib.REDUCE["max"]:
            x, agg = ctx.saved_tensors
            ws_bytes = lib.ngnn_seg_agg_bwd_workspace_bytes(block.n_dst, F, red)
            ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=g.device)
        # algorithmic bytes: gathered grad rows + col_t + degree lookups + rowptr_t + grad_x
        nbytes = block.E * (F * 4 + 4 + 8) + (block.n_src + 1) * 4 + block.n_src * F * 4
        with _timing.span("seg_agg_bwd", nbytes):
            rc = lib.ngnn_seg_agg_bwd(
                _lib.ptr(g), g.stride(0), F, _lib.ptr(block.rowptr), _lib.ptr(block.col),
                block.n_dst, _lib.ptr(t.rowptr), _lib.ptr(t.col), block.n_src, red, _lib.F32,
                _lib.ptr(x), x.stride(0) if x is not None else F,
                _lib.ptr(agg), agg.stride(0) if agg is not None else F,
                _lib.ptr(gx), gx.stride(0), _lib.ptr(ws), ws_bytes, _lib.stream_handle(g.device))
        _lib.check(rc, "ngnn_seg_agg_bwd")
        return gx, None, None


def segment_aggregate(x: torch.Tensor, block: Block, reduce: str = "mean") -> torch.Tensor:
    if reduce not in _lib.REDUCE:
        raise ValueError(f"unsupported aggregation {reduce!r} (expected mean, sum/add or max)")
    return _SegmentAggregate.apply(x, block, reduce)
