"""Seed-row cross entropy on the device (ngnn_seed_xent_*).

``seed_cross_entropy(out, y, batch_size)`` == ``F.cross_entropy(out[:batch_size],
y[:batch_size])`` -- the loss of the reference's training loop
(pipeline.py:158) -- in two launches (forward, backward) instead of the
softmax / nll / slice-backward / fill chain.  The input gradient is a
view of a cached buffer whose rows >= batch_size are zero and stay zero (only
rows < batch_size are ever written), and it tells the SAGE stack's backward
how many leading rows can be nonzero (``_ngnn_nonzero_rows``), so that
backward skips its row-extent scan.
"""
from __future__ import annotations

import torch

from . import _lib

_zero_rows: dict = {}
_ws: dict = {}


def _workspace(dev, B: int) -> torch.Tensor:
    """Per-(device, B) loss workspace; zero-filled once (its ticket resets
    itself), then reused by every call on the stream."""
    key = (dev, B)
    buf = _ws.get(key)
    if buf is None:
        n = _lib.load().ngnn_seed_xent_workspace_bytes(B)
        buf = torch.zeros(n, dtype=torch.uint8, device=dev)
        _ws[key] = buf
    return buf


def _grad_buffer(dev, n: int, c: int, b: int) -> torch.Tensor:
    """[n, c] view of a cached zero-initialised buffer; only rows < b are
    ever written, so rows >= b are zero.  Grown on demand (zeros)."""
    key = (dev, c)
    buf = _zero_rows.get(key)
    if buf is None or buf.size(0) < n:
        buf = torch.zeros(max(n, 1), c, dtype=torch.float32, device=dev)
        _zero_rows[key] = buf
    return buf[:n]


class _SeedXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, y, batch_size: int, ignore_index: int):
        B = int(batch_size)
        x = logits if logits.stride(1) == 1 else logits.contiguous()
        yy = y[:B].contiguous()
        loss = torch.empty((), dtype=torch.float32, device=x.device)
        count = torch.empty((), dtype=torch.float32, device=x.device)
        ws = _workspace(x.device, B)
        _lib.check(_lib.load().ngnn_seed_xent_fwd(
            _lib.ptr(x), x.stride(0), B, x.size(1), _lib.ptr(yy), int(ignore_index),
            _lib.ptr(loss), _lib.ptr(count), _lib.ptr(ws), ws.numel(),
            _lib.stream_handle(x.device)), "ngnn_seed_xent_fwd")
        ctx.ws = ws  # holds the row log-sum-exps for the backward (same stream)
        ctx.save_for_backward(x, yy, count)
        ctx.B, ctx.ignore, ctx.n = B, int(ignore_index), logits.size(0)
        return loss

    @staticmethod
    def backward(ctx, g):
        x, yy, count = ctx.saved_tensors
        g = g.contiguous()
        dx = _grad_buffer(x.device, ctx.n, x.size(1), ctx.B)
        _lib.check(_lib.load().ngnn_seed_xent_bwd(
            _lib.ptr(x), x.stride(0), ctx.B, x.size(1), _lib.ptr(yy), ctx.ignore, _lib.ptr(ctx.ws),
            _lib.ptr(g), _lib.ptr(count), _lib.ptr(dx), dx.stride(0), _lib.stream_handle(x.device)),
            "ngnn_seed_xent_bwd")
        dx._ngnn_nonzero_rows = ctx.B  # rows >= B are zero: the SAGE backward's row bound
        return dx, None, None, None


def seed_cross_entropy(logits: torch.Tensor, y: torch.Tensor, batch_size: int,
                       ignore_index: int = -100) -> torch.Tensor:
    """Mean cross entropy of ``logits[:batch_size]`` against ``y[:batch_size]``."""
    if not logits.is_cuda:
        raise RuntimeError("ngnn.losses.seed_cross_entropy: GPU only (no CPU fallback)")
    if logits.dim() != 2 or logits.dtype != torch.float32:
        raise ValueError("logits must be a 2-D float32 tensor")
    if batch_size <= 0 or batch_size > logits.size(0) or y.numel() < batch_size:
        raise ValueError("batch_size out of range")
    return _SeedXent.apply(logits, y, batch_size, ignore_index)
