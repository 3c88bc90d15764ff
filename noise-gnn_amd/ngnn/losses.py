"""Seed-row cross entropy on the device (ngnn_seed_xent_*).

``seed_cross_entropy(out, y, batch_size)`` == ``F.cross_entropy(out[:batch_size],
y[:batch_size])`` -- the loss of the reference's training loop
(pipeline.py:158) -- instead of the softmax / nll / slice-backward / fill
chain.  When the logits need a gradient, ONE launch
(``ngnn_seed_xent_fwd_grad``) writes the loss and the unit-scale gradient;
the backward then costs nothing when its incoming gradient is the training
step's persistent unit tensor (``unit_grad``, marked ``_ngnn_unit``) and one
launch otherwise.  The input gradient is a view of a zero-initialised
buffer whose rows >= batch_size stay zero (only rows < batch_size are ever
written), and it tells the SAGE stack's backward how many leading rows can
be nonzero (``_ngnn_nonzero_rows``), so that backward skips its row-extent
scan.
"""
from __future__ import annotations

import weakref

import torch

from . import _lib

_zero_rows: dict = {}
_ws: dict = {}
_free_grads: dict = {}  # (dev, C, B) -> zero-row gradient buffers not held by a pending node


def unit_grad(loss: torch.Tensor) -> torch.Tensor:
    """A ones tensor shaped like `loss` that the loss backward recognises as 1
    (no scale launch): for a training step's loss.backward(unit_grad(loss)),
    kept by the caller and never modified."""
    one = torch.ones_like(loss)
    one._ngnn_unit = True
    return one


def _take_grad_buffer(dev, n: int, c: int, b: int) -> torch.Tensor:
    """A zero-row [>= n, c] gradient buffer for ONE pending loss node: two
    forwards before one backward (several losses per step) get different
    buffers.  Returned to the pool by the node's backward (or when its graph
    is freed without one)."""
    key = (dev, c, b)
    pool = _free_grads.setdefault(key, [])
    while pool:
        buf = pool.pop()
        if buf.size(0) >= n:
            return buf
    return torch.zeros(max(n, 1), c, dtype=torch.float32, device=dev)


def _give_back(key, buf) -> None:
    _free_grads.setdefault(key, []).append(buf)


class _GradHold:
    """Owns a taken gradient buffer until backward hands it back (weakref
    finalizer: also when the autograd graph is dropped unused)."""

    def __init__(self, key, buf):
        self.buf = buf
        self._fin = weakref.finalize(self, _give_back, key, buf)

    def release(self):
        self._fin()


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
    ever written, so rows >= b are zero.  Grown on demand (zeros).  One
    buffer per (C, b): a buffer shared with a larger b would hold that
    call's stale rows in [b, b_larger)."""
    key = (dev, c, b)
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
        lib = _lib.load()
        ctx.hold = None
        if ctx.needs_input_grad[0]:
            # loss + the unit-scale gradient in one launch
            key = (x.device, x.size(1), B)
            hold = _GradHold(key, _take_grad_buffer(x.device, logits.size(0), x.size(1), B))
            dx = hold.buf
            _lib.check(lib.ngnn_seed_xent_fwd_grad(
                _lib.ptr(x), x.stride(0), B, x.size(1), _lib.ptr(yy), int(ignore_index),
                _lib.ptr(loss), _lib.ptr(count), _lib.ptr(dx), dx.stride(0), _lib.ptr(ws),
                ws.numel(), _lib.stream_handle(x.device)), "ngnn_seed_xent_fwd_grad")
            ctx.hold = hold
        else:
            _lib.check(lib.ngnn_seed_xent_fwd(
                _lib.ptr(x), x.stride(0), B, x.size(1), _lib.ptr(yy), int(ignore_index),
                _lib.ptr(loss), _lib.ptr(count), _lib.ptr(ws), ws.numel(),
                _lib.stream_handle(x.device)), "ngnn_seed_xent_fwd")
        ctx.ws = ws
        ctx.save_for_backward(x, yy, count)
        ctx.B, ctx.ignore, ctx.n = B, int(ignore_index), logits.size(0)
        return loss

    @staticmethod
    def backward(ctx, g):
        x, yy, count = ctx.saved_tensors
        hold = ctx.hold
        if hold is not None:
            # the gradient rows the forward wrote (unit scale); the buffer goes
            # back to the pool -- stream order protects it until its consumer
            # (this backward pass) has read it
            dx = hold.buf[:ctx.n]
            ctx.hold = None
            hold.release()
            if getattr(g, "_ngnn_unit", False):
                dx._ngnn_nonzero_rows = ctx.B  # rows >= B are zero: the SAGE backward's row bound
                return dx, None, None, None
        else:
            dx = _grad_buffer(x.device, ctx.n, x.size(1), ctx.B)
        g = g.contiguous()
        _lib.check(_lib.load().ngnn_seed_xent_bwd(
            _lib.ptr(x), x.stride(0), ctx.B, x.size(1), _lib.ptr(yy), ctx.ignore, _lib.ptr(ctx.ws),
            _lib.ptr(g), _lib.ptr(count), _lib.ptr(dx), dx.stride(0), _lib.stream_handle(x.device)),
            "ngnn_seed_xent_bwd")
        dx._ngnn_nonzero_rows = ctx.B  # rows >= B are zero: the SAGE backward's row bound
        return dx, None, None, None


_bf16_rows: dict = {}


class _SeedXentBF16(torch.autograd.Function):
    """seed_cross_entropy of bf16 logits: only rows < B are widened (B x C, not
    the N x C logits), the fp32 kernels run on them, and the gradient comes
    back as bf16 [N, C] with rows >= B zero (a cached buffer, like the fp32
    path's) carrying the row hint."""

    @staticmethod
    def forward(ctx, logits, y, batch_size: int, ignore_index: int):
        B = int(batch_size)
        ctx.n_full = logits.size(0)
        # the seed rows widened by the library (exact; an ATen copy kernel
        # otherwise), then the fp32 node's forward on them (it fills ctx for
        # its backward: saved rows, ws, B, n = B)
        lw = logits if logits.stride(1) == 1 else logits.contiguous()
        wide = torch.empty(B, lw.size(1), dtype=torch.float32, device=lw.device)
        _lib.check(_lib.load().ngnn_widen_bf16_rows(_lib.ptr(lw), lw.stride(0), lw.size(1), B, None,
                                                    _lib.ptr(wide), wide.stride(0),
                                                    _lib.stream_handle(lw.device)), "ngnn_widen_bf16_rows")
        return _SeedXent.forward(ctx, wide, y, B, ignore_index)

    @staticmethod
    def backward(ctx, g):
        dx, _, _, _ = _SeedXent.backward(ctx, g)  # fp32 [B, C] (ctx.n == B there)
        n, B, C = ctx.n_full, ctx.B, dx.size(1)
        key = (dx.device, C, B, "bf16")
        buf = _bf16_rows.get(key)
        if buf is None or buf.size(0) < n:
            buf = torch.zeros(max(n, 1), C, dtype=torch.bfloat16, device=dx.device)
            _bf16_rows[key] = buf
        out = buf[:n]
        d = dx[:B] if dx[:B].is_contiguous() else dx[:B].contiguous()
        _lib.check(_lib.load().ngnn_cast_f32_bf16(_lib.ptr(d), _lib.ptr(out), B * C,
                                                  _lib.stream_handle(d.device)), "ngnn_cast_f32_bf16")
        out._ngnn_nonzero_rows = B
        return out, None, None, None


class _CastKeepRows(torch.autograd.Function):
    """x.to(dtype) whose backward keeps the nonzero-row hint on the gradient
    (a plain cast's backward returns a fresh tensor without it, and the SAGE
    stack's backward would then bound nothing: every row)."""

    @staticmethod
    def forward(ctx, x, dtype):
        ctx.src = x.dtype
        return x.to(dtype)

    @staticmethod
    def backward(ctx, g):
        gi = g.to(ctx.src)
        rows = getattr(g, "_ngnn_nonzero_rows", None)
        if rows is not None:
            gi._ngnn_nonzero_rows = rows
        return gi, None


def cast_keep_rows(x: torch.Tensor, dtype) -> torch.Tensor:
    return x if x.dtype == dtype else _CastKeepRows.apply(x, dtype)


class _HeadXent(torch.autograd.Function):
    """The loss a graph slot's two-layer forward already took (ngnn.fused.
    LossHead, include/ngnn.h ngnn_xent_head): forward hands its loss over;
    backward, for the training step's unit gradient, hands over the gradient
    rows that forward wrote -- marked with their scatter onto the source rows
    (_ngnn_g_pre), which the stack's backward then skips.  Any other incoming
    gradient: the scaled rows recomputed from the logits (ngnn_seed_xent_bwd)."""

    @staticmethod
    def forward(ctx, logits, res):
        ctx.res = res
        ctx.n = logits.size(0)
        ctx.save_for_backward(logits)
        return res.loss

    @staticmethod
    def backward(ctx, g):
        res = ctx.res
        hd = res.head
        if getattr(g, "_ngnn_unit", False):
            dy = hd.dy[:ctx.n]
            dy._ngnn_nonzero_rows = hd.B
            dy._ngnn_g_pre = hd.g
            return dy, None
        (x,) = ctx.saved_tensors
        dx = _grad_buffer(x.device, ctx.n, x.size(1), hd.B)
        yy = hd.y[:hd.B]
        g = g.contiguous()
        _lib.check(_lib.load().ngnn_seed_xent_bwd(
            _lib.ptr(x), x.stride(0), hd.B, x.size(1), _lib.ptr(yy), hd.ignore, _lib.ptr(hd.ws),
            _lib.ptr(g), _lib.ptr(res.count), _lib.ptr(dx), dx.stride(0), _lib.stream_handle(x.device)),
            "ngnn_seed_xent_bwd")
        dx._ngnn_nonzero_rows = hd.B
        return dx, None


def seed_cross_entropy(logits: torch.Tensor, y: torch.Tensor, batch_size: int,
                       ignore_index: int = -100) -> torch.Tensor:
    """Mean cross entropy of ``logits[:batch_size]`` against ``y[:batch_size]``."""
    if not logits.is_cuda:
        raise RuntimeError("ngnn.losses.seed_cross_entropy: GPU only (no CPU fallback)")
    res = getattr(logits, "_ngnn_head", None)
    if (res is not None and not res.used and logits.dtype == torch.float32 and logits.requires_grad
            and y.data_ptr() == res.head.y.data_ptr() and y.numel() >= batch_size
            and int(batch_size) == res.head.B and int(ignore_index) == res.head.ignore):
        # the slot's forward took this loss already (ngnn.fused.LossHead)
        res.used = True
        return _HeadXent.apply(logits, res)
    if logits.dtype == torch.bfloat16:  # bf16 models: the loss is taken in fp32
        if logits.dim() == 2 and 0 < batch_size <= logits.size(0) and y.numel() >= batch_size:
            return _SeedXentBF16.apply(logits, y, batch_size, ignore_index)
        logits = cast_keep_rows(logits, torch.float32)
    if logits.dim() != 2 or logits.dtype != torch.float32:
        raise ValueError("logits must be a 2-D float32 (or bf16) tensor")
    if batch_size <= 0 or batch_size > logits.size(0) or y.numel() < batch_size:
        raise ValueError("batch_size out of range")
    return _SeedXent.apply(logits, y, batch_size, ignore_index)


# ---------------------------------------------------------------------------
# Co-teaching loss (CTLoss, src/utils/losses.py:10-49) on the device

class _CTState:
    """Outputs of one ngnn_ct_loss_fwd launch pair, shared by the two
    per-model autograd nodes (each model's backward reads the rows the other
    model kept from the workspace)."""
    __slots__ = ("ws", "out", "y_noise", "ignore", "B", "C")


class _CTPick(torch.autograd.Function):
    """loss_m (already computed by the shared forward) as a differentiable
    function of y_m alone, so that loss_1.backward() and loss_2.backward()
    each run only their own model's graph, as in pipeline.py:125-131.
    y_m may hold more rows than the loss reads (the whole block's logits,
    CTLoss(..., batch_size=B)): its gradient is then a zero-row buffer whose
    rows < B the backward launch writes (no slice backward), marked for the
    SAGE stack's bounded backward."""

    @staticmethod
    def forward(ctx, y, state: _CTState, m: int):
        ctx.state, ctx.m, ctx.n = state, m, y.size(0)
        ctx.save_for_backward(y)
        return state.out[m].clone()

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        st = ctx.state
        if ctx.n > st.B:  # rows >= B never written: zero (one buffer per model)
            dy = _grad_buffer(y.device, ctx.n, st.C, ("ct", ctx.m, st.B))
        else:
            dy = torch.empty(st.B, st.C, dtype=torch.float32, device=y.device)
        g = g.reshape(1).to(torch.float32).contiguous()
        _lib.check(_lib.load().ngnn_ct_loss_bwd(
            ctx.m, _lib.ptr(y), y.stride(0), st.B, st.C, _lib.ptr(st.y_noise), st.ignore,
            _lib.ptr(st.ws), _lib.ptr(g), _lib.ptr(dy), dy.stride(0),
            _lib.stream_handle(y.device)), "ngnn_ct_loss_bwd")
        dy._ngnn_nonzero_rows = st.B
        return dy, None, None


class CTLoss(torch.nn.Module):
    """Drop-in for the reference's ``CTLoss(device)`` (losses.py:10-49).

    ``forward(y_1, y_2, y_noise, forget_rate, ind, noise_or_not)`` returns the
    same 8-tuple ``(loss_1_update, loss_2_update, pure_ratio_1, pure_ratio_2,
    ind_1_update, ind_2_update, ind_noisy_1, ind_noisy_2)`` with no host
    round trip: the per-row cross entropies, both argsorts, the exchange
    selection and the pure ratios are two device launches
    (``ngnn_ct_loss_fwd``), each loss's backward one launch.

    Differences from the reference, all documented in DESIGN.md: the index
    outputs are device int64 tensors instead of numpy arrays (the pipelines
    discard them, pipeline.py:116); tied losses are ordered by row index
    (np.argsort's quicksort leaves ties unspecified); ``noise_or_not`` is
    best passed as a device bool tensor (a CPU one is copied per call);
    batches of at most 8192 rows.
    """

    def __init__(self, device=None, ignore_index: int = -100):
        super().__init__()
        self.device = device
        self.ignore_index = ignore_index
        # device int32: nonzero once an `ind` entry fell outside noise_or_not
        # (the reference raises IndexError there; checking it needs a sync)
        self.index_error = None

    def forward(self, y_1, y_2, y_noise, forget_rate, ind, noise_or_not, batch_size: int | None = None):
        """batch_size (extension): y_1 / y_2 are a block's whole logits [N, C]
        and the loss reads rows < batch_size -- the reference's
        ``model(x, ei)[:batch_size]`` without the slice (pipeline.py:113-114);
        each model's gradient then comes back [N, C], zero past the seeds."""
        if not (y_1.is_cuda and y_2.is_cuda):
            raise RuntimeError("ngnn.losses.CTLoss: GPU only (no CPU fallback)")
        if y_1.dim() != 2 or y_1.shape != y_2.shape or y_1.dtype != torch.float32 \
                or y_2.dtype != torch.float32:
            raise ValueError("y_1, y_2 must be float32 [B, C] tensors of the same shape")
        B, C = y_1.shape
        if batch_size is not None:
            if not 0 < int(batch_size) <= B:
                raise ValueError(f"batch_size {batch_size} outside (0, {B}]")
            B = int(batch_size)
        dev = y_1.device
        remember_rate = 1 - forget_rate
        num_remember = int(remember_rate * B)  # losses.py:29-30, same float arithmetic
        if not 0 <= num_remember <= B:
            raise ValueError(f"forget_rate {forget_rate} gives num_remember {num_remember}")
        a = y_1 if y_1.stride(1) == 1 else y_1.contiguous()
        b = y_2 if y_2.stride(1) == 1 else y_2.contiguous()
        yn = y_noise.to(device=dev, dtype=torch.int64).reshape(-1)
        if batch_size is not None:  # (a block's labels / ids: the seed rows')
            yn = yn[:B]
            ind = None if ind is None else ind.reshape(-1)[:B]
        yn = yn.contiguous()
        if yn.numel() != B:
            raise ValueError("y_noise must hold one label per row")
        idx = None if ind is None else ind.to(device=dev, dtype=torch.int64).contiguous()
        clean = None
        if noise_or_not is not None:
            clean = noise_or_not.to(device=dev, dtype=torch.bool).contiguous()
        # per call (caching allocator, no sync): both backwards read it later
        ws = torch.empty(_lib.load().ngnn_ct_loss_workspace_bytes(B), dtype=torch.uint8, device=dev)
        out = torch.empty(4, dtype=torch.float32, device=dev)
        i1 = torch.empty(B, dtype=torch.int64, device=dev)
        i2 = torch.empty(B, dtype=torch.int64, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        _lib.check(_lib.load().ngnn_ct_loss_fwd(
            _lib.ptr(a), a.stride(0), _lib.ptr(b), b.stride(0), B, C, _lib.ptr(yn),
            int(self.ignore_index), num_remember, _lib.ptr(idx), _lib.ptr(clean),
            0 if clean is None else clean.numel(), _lib.ptr(out), _lib.ptr(i1), _lib.ptr(i2),
            _lib.ptr(ws), ws.numel(), _lib.ptr(err), _lib.stream_handle(dev)), "ngnn_ct_loss_fwd")
        self.index_error = err
        st = _CTState()
        st.ws, st.out, st.y_noise, st.ignore, st.B, st.C = ws, out, yn, int(self.ignore_index), B, C
        loss_1 = _CTPick.apply(a, st, 0)
        loss_2 = _CTPick.apply(b, st, 1)
        return (loss_1, loss_2, out[2], out[3], i1[:num_remember], i2[:num_remember],
                i1[num_remember:], i2[num_remember:])
