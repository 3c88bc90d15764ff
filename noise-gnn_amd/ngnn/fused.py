"""Whole-stack SAGE forward/backward on the fused kernels (no host syncs).

``SAGE.forward`` (sage.py:30-40) runs, per layer, ``conv -> relu -> dropout``.
Here one autograd node covers the whole stack.

forward, per layer — ``ngnn_sage_fwd``: gather-aggregate + fp32 MFMA for
``[x | agg] . [W_r; W_l]^T + b`` + ReLU + dropout (hash RNG) in ONE launch.
The aggregate of rows that have in-edges is saved as a side output for the
weight gradient (no re-gather in backward).

backward — every reference pipeline trains on ``out[:batch_size]``
(pipeline.py:155), so the output gradient is zero past row R.  The bounds
live on the DEVICE: ``ngnn_row_extent`` writes R for the top layer, and per
layer ``ngnn_block_prefix_stats`` writes R' = max(R, 1 + max source of the
edges into rows < R) for the layer below.  Per layer:

* ``ngnn_sage_wgrad``: dW_r, dW_l, db over rows < R (ReLU/dropout backward
  fused into the staging of dz), fixed-order reduction;
* input gradient (MEAN/SUM, Fo < K, the default): ``ngnn_sage_dgrad_lowdim``
  scatters dz in the narrow Fo-wide space, then one MFMA pass writes
  dh = dz W_r + g W_l for rows < R'; otherwise ``ngnn_sage_dgrad_fused``
  (per-row products + K-wide atomics), or in deterministic mode
* ``ngnn_sage_fwd`` in dgrad mode: [dz W_l | dz W_r] for rows < R;
* ``ngnn_sage_dgrad_gather``: input gradient rows < R' = root term + the
  transposed aggregation over the source-grouped CSR (edges into rows >= R
  skipped).

Skipped rows contribute exact zeros, so the result equals the dense autograd
graph's up to fp32 summation order; nothing is read back to the host.
"""
from __future__ import annotations

import ctypes
import os
import weakref

import torch

from . import _eager, _lib, _timing
from .block import Block

_ws: dict = {}

# Root-term arithmetic of the fused layer forward (include/ngnn.h,
# NGNN_MATH_EXACT_F32).  False (default): fp32-accurate 3 x bf16 split MFMA --
# error below the fp32 rounding of the reference's own GEMM (DESIGN.md
# section 3).  True: exact fp32 MFMA (a fmaf chain), like torch.backends'
# allow_tf32 = False.
_exact_f32 = False
MFMA_F32_TFS = 157.3  # dense f32 MFMA peak, MI355X (MI355X_MICROARCH.md); bf16 is 16x


def _pad16(n: int) -> int:
    return -(-n // 16) * 16
# debug hook (None in normal use): a list receives (layer, d output, saved
# aggregate) from every fused-stack backward
_debug_grads = None
# test hook: when a list, every stack forward appends fp32 clones of its hidden
# activations (inside a capture the clones replay with the step) -- the oracle
# tests take the GPU's ReLU decision where a pre-activation sits at the kink
_debug_acts = None


def dropout_scale(p: float) -> float:
    """The fused kernels' survivor scale (ngnn_device.h Dropout): p is
    resolved to p_eff = ceil(p * 256) / 256 and survivors scale by
    1 / (1 - p_eff) (fp32), so the expectation is exact."""
    import math
    import numpy as np
    pf = float(np.float32(p))
    if pf <= 0.0:
        return 1.0
    t = max(1, min(256, math.ceil(pf * 256.0)))
    return 0.0 if t >= 256 else float(np.float32(256.0) / np.float32(256 - t))


def set_exact_f32(flag: bool) -> None:
    global _exact_f32
    _exact_f32 = bool(flag)


class exact_f32:
    """Context manager: exact fp32 MFMA for the layer forward inside it."""

    def __init__(self, flag: bool = True):
        self.flag = flag

    def __enter__(self):
        global _exact_f32
        self.prev, _exact_f32 = _exact_f32, self.flag
        return self

    def __exit__(self, *exc):
        global _exact_f32
        _exact_f32 = self.prev
        return False


# superseded workspaces, kept alive: a captured HIP graph holds the raw
# address of the buffer it was captured with, so a later, larger eager call
# must never free it (the replays would write into memory the caching
# allocator has handed on -- ADVICE r4).  Growth is rare (sizes follow the
# largest block seen); the list only ever holds the smaller generations.
_ws_retired: list = []


def _workspace(dev: torch.device, name: str, nbytes: int, zero: bool = False) -> torch.Tensor:
    """Per-device scratch buffers, grown on demand and reused across calls
    (stream-ordered).  zero: zero-filled when (re)allocated.  A grown
    buffer's predecessor is retired, not freed (graph captures may hold it)."""
    key = (dev, name)
    buf = _ws.get(key)
    if buf is None or buf.numel() < nbytes:
        alloc = torch.zeros if zero else torch.empty
        if buf is not None:
            _ws_retired.append(buf)
        buf = alloc(max(nbytes, 256), dtype=torch.uint8, device=dev)
        _ws[key] = buf
    return buf


def pack_weight(w: torch.Tensor) -> torch.Tensor:
    Fo, K = w.shape
    lib = _lib.load()
    packed = torch.empty(lib.ngnn_pack_weight_bytes(Fo, K) // 4, dtype=torch.float32,
                         device=w.device)
    w = w.detach()
    if w.stride(1) != 1:
        w = w.contiguous()
    _lib.check(lib.ngnn_pack_weight(_lib.ptr(w), w.stride(0), Fo, K, _lib.ptr(packed),
                                    _lib.stream_handle(w.device)), "ngnn_pack_weight")
    return packed


def pack_dgrad_weight(wl: torch.Tensor, wr: torch.Tensor) -> torch.Tensor:
    """Fragment-packed [W_l^T ; W_r^T]  ([2K x Fo]) for dz -> [dz W_l | dz W_r]."""
    Fo, K = wl.shape
    lib = _lib.load()
    wl, wr = wl.detach().contiguous(), wr.detach().contiguous()
    packed = torch.empty(lib.ngnn_pack_weight_bytes(2 * K, Fo) // 4, dtype=torch.float32,
                         device=wl.device)
    _lib.check(lib.ngnn_pack_weight_ex(_lib.ptr(wl), _lib.ptr(wr), K, K, 2 * K, Fo, 1,
                                       _lib.ptr(packed), _lib.stream_handle(wl.device)),
               "ngnn_pack_weight_ex")
    return packed


def _gemm_layer(x, K, n_rows, block, reduce, pl, pr, bias, Fo, out, relu, p_drop, seed,
                agg_out=None, n_rows_dev=None, xmask=None, xscale=1.0, seed_dev=None):
    if torch.is_tensor(n_rows_dev):
        n_rows_dev = _lib.ptr(n_rows_dev)
    rc = _lib.load().ngnn_sage_fwd(
        _lib.ptr(x), x.stride(0), K, n_rows, n_rows_dev,
        _lib.ptr(block.rowptr) if block is not None else None,
        _lib.ptr(block.col) if block is not None else None,
        _lib.REDUCE[reduce], _lib.ptr(pl), _lib.ptr(pr), _lib.ptr(bias), Fo, _lib.ptr(out),
        out.stride(0), int(relu), float(p_drop), seed & (2**64 - 1), _lib.ptr(seed_dev),
        _lib.ptr(agg_out), agg_out.stride(0) if agg_out is not None else K,
        _lib.ptr(xmask), xmask.stride(0) if xmask is not None else K, float(xscale),
        _lib.stream_handle(x.device))
    _lib.check(rc, "ngnn_sage_fwd")


def narrow_ok(reduce: str, K: int, Fo: int, relu: bool, p_drop: float) -> bool:
    """Can this layer aggregate its neighbour term in the F_out-wide space
    (NGNN_FWD_NARROW)?  A linear aggregation into a narrower output layer
    with no epilogue beyond the bias, on the split-MFMA path, with both
    weight halves in one LDS image (2 ceil(F_out/16) <= 6 tiles)."""
    return (reduce in ("mean", "sum") and not relu and p_drop == 0.0 and Fo < K
            and -(-Fo // 16) <= 3 and not _exact_f32)


def sage_layer_fwd(x: torch.Tensor, block: Block, reduce: str, wl, bl, wr, relu: bool,
                   p_drop: float, seed: int, agg_out: torch.Tensor | None = None,
                   seed_dev: torch.Tensor | None = None,
                   x_dev: torch.Tensor | None = None, span: str = "sage_fwd",
                   narrow: bool = False, xrow_dev: torch.Tensor | None = None,
                   x_rows: int = 0, w_bf16: bool = False,
                   wl_packed: torch.Tensor | None = None, out_bf16: bool = False) -> torch.Tensor:
    """One fused SAGEConv(+relu+dropout) layer, no autograd.  x_dev: device
    word holding the address of x's rows (zero-copy graph slot); x then only
    supplies the shape.  xrow_dev (with x_dev): device word holding the
    address of the block's n_id when x_dev points at the whole x_rows-row
    feature table (fused x[n_id] gather; 0 at run time: plain rows).
    narrow: aggregate the neighbour term as mean/sum of z = x W_l^T (F_out
    wide) instead of x (K wide) -- the output layer's form (no agg_out then).
    w_bf16: the weights hold bf16-exact values (a bf16 model's parameters,
    widened): NGNN_W_BF16, a one-part split image (same sums, fewer MFMAs and
    wider column slices).  wl_packed: ngnn_pack_weight(wl) kept current by a
    producer (NGNN_WL_PREPACKED: no pack launch when W_l streams from L2).
    out_bf16: return bf16 rows (NGNN_OUT_BF16, a bf16 model's hidden
    activations, rounded in the epilogue); fp32 when the layer's kernel
    cannot (narrow / wide / partial 16-column tiles)."""
    N, K = x.shape
    Fo = wl.shape[0]
    if x.dtype == torch.bfloat16 and (not bf16_rows_ok(x, narrow) or (
            x_dev is None and _lib.load().ngnn_sage_wide_preferred(K, Fo, int(_exact_f32)))):
        # (the wide path reads fp32 rows: bf16 rows widened, exactly)
        x = x.float()
    xb = x.dtype == torch.bfloat16  # bf16 rows read as such (NGNN_X_BF16)
    out_bf16 = out_bf16 and not narrow and Fo % 16 == 0
    out = torch.empty(N, Fo, dtype=torch.bfloat16 if out_bf16 else torch.float32, device=x.device)
    root = wr is not None  # (None: GCNConv's aggregate-first form, no root term)
    # algorithmic bytes: x + gathered rows + col + rowptr + out;  flops: root GEMM on
    # every row + neighbour GEMM on rows with in-edges (0 if not known: conservative)
    nbytes = ((N * K + block.E * K) * (2 if xb else 4) + block.E * 4 + N * Fo * (2 if out_bf16 else 4)
              + (N + 1) * 4)
    n_e = int(block.n_active or 0)
    flops = 2 * N * K * Fo * root + 2 * n_e * K * Fo
    # ideal matrix-core time of the instruction mix: the
    # root term on 6 bf16 products per fp32 product (bf16 dense 16x the f32
    # MFMA rate) unless exact, the neighbour term on f32 MFMA
    w1 = w_bf16 and not _exact_f32 and reduce != "max"
    # bf16 products per fp32 product of the root term: 6 (3 with bf16 rows);
    # one-part weights: 3 (1 with bf16 rows)
    nprod = (1 if xb else 3) if w1 else (3 if xb else 6)
    root_rate = MFMA_F32_TFS * 1e12 * (1.0 if _exact_f32 else 16.0 / nprod)
    mfma_s = 2 * N * K * Fo * root / root_rate + 2 * n_e * K * Fo / (MFMA_F32_TFS * 1e12)
    if xrow_dev is not None:  # the n_id loads of the fused gather (rows, neighbours)
        nbytes += (N + block.E) * 8
    if narrow and agg_out is None:
        # narrow mode: the root launch also computes z = x W_l^T (every row),
        # then gathers z (F_out wide) instead of x
        nbytes = (N * K + N * Fo + N * _pad16(Fo) + block.E * (_pad16(Fo) + 1)) * 4 + (N + 1) * 4
        flops = 4 * N * K * Fo
        mfma_s = 4 * N * K * Fo / root_rate
    wl_ = wl.detach()
    wr_ = wr.detach() if root else None
    if wl_.stride(1) != 1 or (root and (wr_.stride(1) != 1 or wl_.stride(0) != wr_.stride(0))):
        wl_, wr_ = wl_.contiguous(), (wr_.contiguous() if root else None)
    xk = x
    if K % 4 and not xb and pad_k_ok(K, Fo) and x_dev is None and not narrow and (
            agg_out is None or agg_out.stride(0) % 4 == 0):
        # the row-tile kernel reads 16-B column quads: one zero column (or
        # three) appended to x and to the weights -- 0 * 0 terms, the same
        # sums -- instead of the 64-row fallback (Amazon-Computers' K = 767)
        K4 = K + (-K) % 4
        xk = torch.zeros(N, K4, dtype=torch.float32, device=x.device)
        xk[:, :K].copy_(x)
        wl_ = _pad_cols(wl_, K4)
        wr_ = _pad_cols(wr_, K4) if root else None
    nrd = _lib.ptr(block.n_rows_dev) if block.n_rows_dev is not None else None
    lib = _lib.load()
    if (not xb and xrow_dev is None and not (narrow and agg_out is None)
            and lib.ngnn_sage_wide_preferred(xk.size(1), Fo, int(_exact_f32))):
        # the wide path (ngnn_wide.hip): exact f32 MFMA throughout, and the
        # aggregate of the rows with in-edges written then re-read
        mfma_s = flops / (MFMA_F32_TFS * 1e12)
        nbytes += 2 * n_e * K * 4
    ws = _workspace(x.device, "sage_fwd", lib.ngnn_sage_fwd_raw_workspace_bytes(K, Fo, N), zero=True)
    prepacked = 0
    if (wl_packed is not None and not narrow and xk is x and wl_.data_ptr() == wl.data_ptr()
            and wl_packed.numel() * 4 >= lib.ngnn_pack_weight_bytes(Fo, K)):
        ws, prepacked = wl_packed, _lib.WL_PREPACKED
    with _timing.span(span, nbytes, flops, mfma_s) as rec:
        # raw weights straight into the row-tile kernel; packed fallback otherwise
        # rows >= n_active have no in-edges (a sampler-built block): dense kernel
        n_edge = N if block.n_active is None else min(int(block.n_active), N)
        rc = lib.ngnn_sage_fwd_raw(
            _lib.ptr(xk), _lib.ptr(x_dev), None, _lib.ptr(xrow_dev), int(x_rows), xk.stride(0),
            xk.size(1), N, nrd, n_edge,
            _lib.ptr(block.n_edge_rows_dev), _lib.ptr(block.rowptr), _lib.ptr(block.col),
            _lib.ptr(block.col_x) if xrow_dev is not None else None,
            _lib.REDUCE[reduce] | (_lib.MATH_EXACT_F32 if _exact_f32 else 0)
            | (_lib.FWD_NARROW if (narrow and agg_out is None) else 0)
            | (_lib.X_BF16 if xb else 0) | (_lib.W_BF16 if w1 else 0) | prepacked
            | (_lib.OUT_BF16 if out_bf16 else 0),
            _lib.ptr(wl_), _lib.ptr(wr_), wl_.stride(0), _lib.ptr(bl), Fo,
            _lib.ptr(out), out.stride(0), int(relu), float(p_drop), seed & (2**64 - 1),
            _lib.ptr(seed_dev), _lib.ptr(agg_out),
            agg_out.stride(0) if agg_out is not None else xk.size(1),
            _lib.ptr(ws), ws.numel() * ws.element_size(), _lib.stream_handle(x.device))
        if rc == _lib.E_SHAPE and out_bf16:
            # this layer's kernel writes fp32 rows only
            return sage_layer_fwd(x, block, reduce, wl, bl, wr, relu, p_drop, seed, agg_out,
                                  seed_dev, x_dev, span, narrow, xrow_dev, x_rows, w_bf16,
                                  wl_packed, out_bf16=False)
        if rc == _lib.E_SHAPE and xb and x_dev is None:
            # bf16 rows outside the bf16 envelope: the fp32 path on widened rows
            return sage_layer_fwd(x.float(), block, reduce, wl, bl, wr, relu, p_drop, seed,
                                  agg_out, seed_dev, None, span, narrow, w_bf16=w_bf16)
        if rc == _lib.E_SHAPE:
            if x_dev is not None:
                raise _lib.NGNNError("zero-copy input outside the row-tile kernel's envelope")
            if rec is not None:  # the 64-row kernel is exact fp32 MFMA throughout
                rec.mfma_s = flops / (MFMA_F32_TFS * 1e12)
            pl = pack_weight(wl)
            pr = pack_weight(wr if root else _zeros_like_cached(wl))
            _gemm_layer(x, K, N, block, reduce, pl, pr, bl, Fo, out, relu, p_drop, seed,
                        agg_out=agg_out, seed_dev=seed_dev, n_rows_dev=block.n_rows_dev)
        else:
            _lib.check(rc, "ngnn_sage_fwd_raw")
    return out


def bf16_rows_ok(x: torch.Tensor, narrow: bool = False) -> bool:
    """Can the row-tile kernel read these bf16 rows directly (NGNN_X_BF16)?
    Split-bf16 root term (not the exact-fp32 mode), rows of a multiple of 4
    elements on 8-B boundaries, a 16-B aligned base (narrow layers too: the
    output layer reading a bf16 model's hidden activations)."""
    return (x.dtype == torch.bfloat16 and not _exact_f32 and x.dim() == 2
            and x.stride(1) == 1 and x.size(1) % 4 == 0 and x.stride(0) % 4 == 0
            and x.data_ptr() % 16 == 0)


def pad_k_ok(K: int, Fo: int = 0) -> bool:
    """Does a K % 4 != 0 layer run well on the row-tile kernel after padding
    K to a multiple of 4?  Its split-bf16 W_r image (3 x ceil(K/32) KiB per
    16 outputs) must fit the LDS for enough output tiles that F_out takes at
    most two column slices (each slice re-reads x: measured on
    Amazon-Computers' 767 -> 512 layer, 16 slices ran 1.4x slower than the
    64-row kernel)."""
    K4 = K + (-K) % 4
    img = 3 * (-(-K4 // 32)) * 1024
    ntw = next((c for c in (16, 8, 6, 4, 3, 2) if c * img <= 160 * 1024 - 1280), 0)
    return ntw > 0 and -(-Fo // (16 * ntw)) <= 2


def agg_buffer(N: int, K: int, device, Fo: int = 0) -> torch.Tensor:
    """[N, K] saved-aggregate buffer; rows padded to a multiple of 4 floats
    when the forward pads K (pad_k_ok), so the kernel can write it whole."""
    if K % 4 and pad_k_ok(K, Fo):
        K4 = K + (-K) % 4
        return torch.empty(N, K4, dtype=torch.float32, device=device)[:, :K]
    return torch.empty(N, K, dtype=torch.float32, device=device)


def _pad_cols(w: torch.Tensor, K4: int) -> torch.Tensor:
    out = torch.zeros(w.shape[0], K4, dtype=torch.float32, device=w.device)
    out[:, :w.shape[1]].copy_(w)
    return out


def _zeros_like_cached(w: torch.Tensor) -> torch.Tensor:
    """A persistent zero matrix shaped like w (GCN layers' W_r = 0)."""
    key = (w.device, "zeros", tuple(w.shape))
    z = _ws.get(key)
    if z is None:
        z = torch.zeros(w.shape, dtype=torch.float32, device=w.device)
        _ws[key] = z
    return z


def gcn_transform_first(x, block: Block, w, b, relu: bool, p_drop: float, seed: int,
                        seed_dev=None, x_dev=None, span: str = "gcn_fwd", xrow_dev=None,
                        x_rows: int = 0):
    """GCNConv(normalize=False) layer in PyG's own order (convolution.py:19-35,
    GCNConv [ext]): z = x W^T on the row-tile kernel (no bias, no epilogue),
    then ngnn_gcn_agg_fwd: out = act(sum_{j->i} z_j + b) -- the form for
    F_in > F_out (the gather runs at the narrower width)."""
    if x.dtype != torch.float32:  # this launch reads fp32 rows (no NGNN_X_BF16 here)
        if x_dev is not None:
            raise _lib.NGNNError("transform-first GCN layer on a zero-copy non-fp32 input")
        x = x.float()
    N, K = x.shape
    Fo = w.shape[0]
    ldz = _pad16(Fo)
    lib = _lib.load()
    z = _workspace(x.device, "gcn_z", N * ldz * 4).view(torch.float32)[:N * ldz].view(N, ldz)
    wd = w.detach() if w.stride(1) == 1 else w.detach().contiguous()
    ws = _workspace(x.device, "sage_fwd", lib.ngnn_sage_fwd_raw_workspace_bytes(K, Fo, N), zero=True)
    nrd = _lib.ptr(block.n_rows_dev) if block.n_rows_dev is not None else None
    out = torch.empty(N, Fo, dtype=torch.float32, device=x.device)
    root_rate = MFMA_F32_TFS * 1e12 * (1.0 if _exact_f32 else 16.0 / 6.0)
    with _timing.span(span + "_z", (N * K + N * ldz) * 4, 2 * N * K * Fo, 2 * N * K * Fo / root_rate):
        rc = lib.ngnn_sage_fwd_raw(
            _lib.ptr(x), _lib.ptr(x_dev), None, _lib.ptr(xrow_dev), int(x_rows), x.stride(0), K, N,
            nrd, N, None, _lib.ptr(block.rowptr),
            _lib.ptr(block.col), None, _lib.REDUCE["sum"] | (_lib.MATH_EXACT_F32 if _exact_f32 else 0),
            None, _lib.ptr(wd), wd.stride(0), None, Fo, _lib.ptr(z), ldz, 0, 0.0, 0, None, None, K,
            _lib.ptr(ws), ws.numel(), _lib.stream_handle(x.device))
        if rc == _lib.E_SHAPE:
            if x_dev is not None:
                raise _lib.NGNNError("zero-copy input outside the row-tile kernel's envelope")
            _gemm_layer(x, K, N, None, "sum", None, pack_weight(w), None, Fo, z, False, 0.0, 0,
                        n_rows_dev=block.n_rows_dev)
        else:
            _lib.check(rc, "ngnn_sage_fwd_raw")
    with _timing.span(span + "_agg", (block.E * (ldz + 1) + N * Fo) * 4 + (N + 1) * 4):
        _lib.check(lib.ngnn_gcn_agg_fwd(
            _lib.ptr(z), ldz, Fo, _lib.ptr(block.rowptr), _lib.ptr(block.col), N, nrd, _lib.ptr(b),
            int(relu), float(p_drop), seed & (2**64 - 1), _lib.ptr(seed_dev), _lib.ptr(out),
            out.stride(0), _lib.stream_handle(x.device)), "ngnn_gcn_agg_fwd")
    return out


def const_bounds(dev, L: int, R: int) -> torch.Tensor:
    """The stack backward's read-only row-bound array (L + 1 words = R), cached
    per (device, L, R).  A graph producer creates it BEFORE capture (else the
    first captured backward records its fill as a node of every replay)."""
    key = (dev, "bnd", L, int(R))
    bnd = _ws.get(key)
    if bnd is None:
        bnd = torch.full((L + 1,), int(R), dtype=torch.int32, device=dev)
        _ws[key] = bnd
    return bnd


def _dgrad_fused_ok(Fo: int, K: int) -> bool:
    """ngnn_sage_dgrad_fused (per target row, VALU products, W_r and W_l in
    LDS) only while both weights fit its LDS: a wave re-reads the whole of W
    for every row, so with W streamed from L2 (the 3-layer products hidden
    layer, 256 x 256: 512 KiB per row) it ran 845 us/step.  Wider layers take
    the dgrad GEMM (MFMA, rows < R) + scatter."""
    return Fo <= 512 and 2 * Fo * K * 4 + 4 * 512 * 4 <= 150 * 1024


# the two-layer weight-stationary forward (ngnn_sage2_fwd) for the shapes it
# covers; False: always the per-layer kernels (A/B switch, tests)
_use_fwd2 = True


def sage2_ok(x, block: Block, reduce: str, params, w_bf16: bool) -> bool:
    """Does ngnn_sage2_fwd cover this stack?  SAGE(K0, 256, F1) with two
    layers, mean/sum, fp32 rows and weights, a block whose rows with in-edges
    are known to come first (a NeighborLoader block: hinted n_active or the
    graph slot's device word); plain rows or the slot's fused x[n_id]."""
    if not _use_fwd2 or _exact_f32 or w_bf16 or len(params) != 6 or reduce not in ("mean", "sum"):
        return False
    if any(q is None or q.dtype != torch.float32 for q in params):
        return False
    if x.dtype != torch.float32 or x.dim() != 2 or x.stride(1) != 1 or x.stride(0) % 4:
        return False
    if block.n_active is None and block.n_edge_rows_dev is None:
        return False
    wl0, _, wr0, wl1, _, wr1 = params
    if wl0.shape != wr0.shape or wl1.shape != wr1.shape or wl1.shape[1] != wl0.shape[0]:
        return False
    key = (x.size(1), wl0.shape[0], wl1.shape[0], reduce)
    ok = _sage2_supported.get(key)
    if ok is None:  # (a pure function of the shape: asked once -- the eager step is host-bound)
        ok = _sage2_supported[key] = bool(_lib.load().ngnn_sage2_supported(
            x.size(1), wl0.shape[0], wl1.shape[0], _lib.REDUCE[reduce]))
    return ok


_sage2_supported: dict = {}
_ws_bytes: dict = {}


def _ws_size(fn: str, *args) -> int:
    """A workspace-size query of the C ABI (a pure function of its
    arguments), memoised: the eager training step is host-bound."""
    key = (fn,) + args
    v = _ws_bytes.get(key)
    if v is None:
        v = _ws_bytes[key] = int(getattr(_lib.load(), fn)(*args))
    return v


def fwd2_fused() -> bool:
    """Does ngnn_sage2_fwd run its edge and main stages as ONE launch
    (k_fwd2x; NGNN_FWD2_FUSE=0 keeps two -- read by the library once)?"""
    return os.environ.get("NGNN_FWD2_FUSE", "1") != "0"


def sage2_params(params):
    """The six tensors ngnn_sage2_fwd / _bwd take.  A two-layer SimpleGCN
    stack ([W, b, None] per GCNConv(normalize=False), sum aggregation) is the
    SAGE stack with W_r = 0 (convolution.py:29-35): its absent root weights
    become persistent zero matrices -- the root products add exact zeros and
    their gradients go to scratch (_absent_none drops them).  A stack with
    only one absent W_r: None (not this path)."""
    if params[2] is None and params[5] is None and params[0] is not None and params[3] is not None:
        return [params[0], params[1], _zeros_like_cached(params[0]),
                params[3], params[4], _zeros_like_cached(params[3])]
    if any(q is None for q in params):
        return None
    return list(params)


def _absent_none(params, grads):
    """The gradients of the stack's parameters: None where the caller's
    parameter is absent (a GCN layer's W_r, sage2_params)."""
    return [None if q is None else g for q, g in zip(params, grads)]


def sage2_forward(x, block: Block, reduce: str, params, p_drop: float, seed: int, seed_dev,
                  stages: int | None = None, bufs=None, head: "HeadResult | None" = None,
                  root0: bool = True):
    """(h, logits, layer-0 aggregate, h partial?) of a two-layer stack in one
    call (include/ngnn.h ngnn_sage2_fwd).  h holds the rows the bounded
    backward reads: every row, or rows < R' when the graph slot vouches that
    the loss reads rows < its B (block.r_next[2]).  stages / bufs (bench.py's
    per-launch timing): a subset of the launches, on the (h, out, agg0) of an
    earlier call.  head: this forward's loss head (LossHead.start), or None.
    root0 False: layer 0 has no root term (a SimpleGCN stack, sage2_params'
    zero W_r0): the kernels skip x entirely (ABI 17, wr0 NULL) -- not with the
    fused x[n_id] gather, which keeps the zero matrix."""
    # (pointers and strides only: no detach -- nothing here records autograd)
    wl0, bl0, wr0, wl1, bl1, wr1 = params
    if wl0.stride(1) != 1 or wr0.stride(0) != wl0.stride(0) or wr0.stride(1) != 1:
        wl0, wr0 = wl0.contiguous(), wr0.contiguous()
    if wl1.stride(1) != 1 or wr1.stride(0) != wl1.stride(0) or wr1.stride(1) != 1:
        wl1, wr1 = wl1.contiguous(), wr1.contiguous()
    bl0, bl1 = bl0.contiguous(), bl1.contiguous()
    N, K0 = x.shape
    H, F1 = wl0.shape[0], wl1.shape[0]
    dev = x.device
    lib = _lib.load()
    if bufs is None:
        h = torch.empty(N, H, dtype=torch.float32, device=dev)
        out = torch.empty(N, F1, dtype=torch.float32, device=dev)
        agg0 = agg_buffer(N, K0, dev, H)
    else:
        h, out, agg0 = bufs[:3]
    ws = _workspace(dev, "sage2", _ws_size("ngnn_sage2_workspace_bytes", K0, F1, N))
    n_edge = N if block.n_active is None else min(int(block.n_active), N)
    rn = block.r_next
    h_rows_dev = rn[0] if (rn is not None and len(rn) > 2 and rn[2]) else None
    n_e = int(block.n_active or 0)
    args = [_lib.ptr(x), _lib.ptr(block.x_dev), None, _lib.ptr(block.xrow_dev), int(block.x_rows),
            x.stride(0), K0, N, _lib.ptr(block.n_rows_dev), n_edge, _lib.ptr(block.n_edge_rows_dev),
            _lib.ptr(block.rowptr), _lib.ptr(block.col),
            _lib.ptr(block.col_x) if block.xrow_dev is not None else None, _lib.REDUCE[reduce], _lib.ptr(wl0), _lib.ptr(bl0),
            _lib.ptr(wr0) if (root0 or block.xrow_dev is not None) else None, wl0.stride(0), H,
            _lib.ptr(wl1), _lib.ptr(bl1), _lib.ptr(wr1), wl1.stride(0), F1, float(p_drop),
            seed & (2**64 - 1), _lib.ptr(seed_dev), _lib.ptr(h), h.stride(0), N,
            _lib.ptr(h_rows_dev), _lib.ptr(agg0), agg0.stride(0), _lib.ptr(out), out.stride(0)]
    tail = [_lib.ptr(ws), ws.numel(), _lib.stream_handle(dev)]
    hp = None if head is None else ctypes.byref(head.struct)
    if stages is not None or not _timing.timing():
        _lib.check(lib.ngnn_sage2_fwd(*args, hp, _lib.SAGE2_ALL if stages is None else stages, *tail),
                   "ngnn_sage2_fwd")
        return h, out, agg0, h_rows_dev is not None
    # timed: one span per launch.  Algorithmic bytes / flops per launch
    # (DESIGN.md section 5b); n_e = rows with in-edges (0 when not told: lower bound)
    C0p = 32 * (-(-K0 // 32))  # K0 padded to the fp16 chunks the MFMAs run
    ldz = 16 * (-(-F1 // 16))
    h_rows = N  # (upper bound: under the slot's bound fewer rows are written)
    f16 = 16 * MFMA_F32_TFS * 1e12  # fp16 MFMA peak; three products per fp32-equivalent product
    edge = ("sage2_edge", _lib.SAGE2_EDGE,
            4 * (block.E * (K0 + 1) + n_e * (K0 + 1) + n_e * K0 + n_e * H),
            2 * n_e * K0 * H, 3 * 2 * n_e * C0p * H / f16)
    rk = 1 if (root0 or block.xrow_dev is not None) else 0  # (root-free: x not read, no layer-0 root products)
    main = ("sage2_fwd", _lib.SAGE2_MAIN,
            4 * (rk * N * K0 + n_e * H + h_rows * H + N * F1 + N * ldz),
            rk * 2 * N * K0 * H + 4 * N * H * F1, 3 * (rk * 2 * N * C0p * H + 2 * N * H * 2 * ldz) / f16)
    if fwd2_fused():
        # one launch for both (k_fwd2x, as in the step): its bytes / flops are
        # the two phases' sums (nb's write and read stay: the main phase reads
        # it back through L2)
        stages = [("sage2_fwd", _lib.SAGE2_EDGE | _lib.SAGE2_MAIN, edge[2] + main[2], edge[3] + main[3],
                   edge[4] + main[4])]
    else:
        stages = [edge, main]
    stages.append(("sage2_narrow", _lib.SAGE2_NARROW, 4 * (block.E * (ldz + 1) + 2 * n_e * F1 + n_e + 1), 0, 0.0))
    for name, st, nbytes, flops, mfma_s in stages:
        with _timing.span(name, nbytes, flops, mfma_s):
            rc = lib.ngnn_sage2_fwd(*args, hp, st, *tail)
        _lib.check(rc, "ngnn_sage2_fwd")
    return h, out, agg0, h_rows_dev is not None


class LossHead:
    """A graph slot's seed-row cross entropy, seed_cross_entropy(out, y, B),
    taken by the two-layer forward's narrow launch from the logits it
    finishes (include/ngnn.h ngnn_xent_head): the loss, the unit-scale
    gradient rows and their scatter onto the source rows -- the loss launch
    and the backward's scatter launch of the step disappear.  Persistent
    buffers made before the capture (nothing allocated or filled inside it):
    dy [n_rows, F1] (rows >= B stay zero), g [n_rows, ceil4(F1)] (rows < R'
    zeroed by the forward's edge launch every step), the hand-off workspace.
    One pending head per slot (the step's one forward)."""

    def __init__(self, y: torch.Tensor, B: int, n_rows: int, F1: int, r_word: torch.Tensor,
                 ignore_index: int = -100):
        dev = y.device
        self.y, self.B, self.ignore, self.n_rows, self.F1 = y, int(B), int(ignore_index), int(n_rows), int(F1)
        self.dy = torch.zeros(self.n_rows, self.F1, dtype=torch.float32, device=dev)
        self.g = torch.zeros(self.n_rows, (self.F1 + 3) & ~3, dtype=torch.float32, device=dev)
        self.ws = torch.zeros(max(_lib.load().ngnn_xent_head_workspace_bytes(self.B), 16), dtype=torch.uint8,
                              device=dev)
        # per-source seed-edge counts (two alternating arrays + the selector
        # word): single-edge sources take a plain row store, not atomics
        self.src_count = torch.zeros(2 * self.n_rows + 1, dtype=torch.int32, device=dev)
        self.r_word = r_word  # the slot's R' word (its low int32 half)

    def start(self) -> "HeadResult":
        """The outputs of one forward's head (fresh loss / count scalars)."""
        return HeadResult(self)


class HeadResult:
    __slots__ = ("head", "loss", "count", "struct", "used")

    def __init__(self, head: LossHead):
        dev = head.y.device
        self.head = head
        self.loss = torch.empty((), dtype=torch.float32, device=dev)
        self.count = torch.empty((), dtype=torch.float32, device=dev)
        self.used = False
        self.struct = _lib.XentHead(
            _lib.ptr(head.y), head.B, head.ignore, _lib.ptr(self.loss), _lib.ptr(self.count),
            _lib.ptr(head.dy), head.dy.stride(0), _lib.ptr(head.g), head.n_rows, _lib.ptr(head.r_word),
            _lib.ptr(head.ws), head.ws.numel(), _lib.ptr(head.src_count))


def head_ok(block: Block, x, params) -> bool:
    """May this forward take the slot's loss head?  (grad mode on -- the
    loss head is a training-step device; the atomics of its scatter are
    not deterministic)."""
    hd = block.loss_head
    if (hd is None or len(params) != 6 or not torch.is_grad_enabled()
            or torch.are_deterministic_algorithms_enabled()):
        return False
    return (x.size(0) == hd.n_rows and params[3].shape[0] == hd.F1 and hd.B <= x.size(0)
            and any(q.requires_grad for q in params if q is not None))


_use_bwd2 = True  # (tests flip it to compare with the per-layer backward)


def reserve_sage2_bwd(dev, n_rows: int, K0: int, F1: int) -> torch.Tensor:
    """ngnn_sage2_bwd's workspace (zero-filled when first made or grown; the
    backward leaves its g part zero).  A graph slot reserves it before its
    capture: a zero fill inside the captured step would replay every step."""
    lib = _lib.load()
    return _workspace(dev, ("sage2_bwd", K0, F1), _ws_size("ngnn_sage2_bwd_workspace_bytes", n_rows, K0, F1),
                      zero=True)


# the graph slot's Adam step folded into the two-layer backward's reduction
# (include/ngnn.h ngnn_adam_fold): set by GraphedTrainStep around its capture
# only -- an eager backward never updates parameters
_adam_fold = None


class AdamFoldSpec:
    """ngnn.optim.Adam's step for the six tensors of a two-layer stack,
    taken by ngnn_sage2_bwd's reduction (one launch less per step).  used:
    set when a captured backward took it (the slot then captures no
    optimizer launch)."""

    def __init__(self, opt, params):
        st = opt.state
        group = opt.param_groups[0]
        step = st[params[0]]["step"]
        # [W_l0, b0, W_r0, W_l1, b1, W_r1] (the stack's order; a GCN stack's
        # absent W_r: the zero matrices its forward reads, sage2_params)
        self.params = sage2_params(params)
        b1, b2 = group["betas"]
        # the update of an absent W_r lands in scratch tensors of its shape
        # (never in the zeros the forward reads)
        slots = []
        self._scratch = []
        for q, z in zip(params, self.params):
            if q is None:
                t = torch.zeros(3, *z.shape, dtype=torch.float32, device=z.device)
                self._scratch.append(t)
                slots.append((t[0], t[1], t[2]))
            else:
                slots.append((q, st[q]["exp_avg"], st[q]["exp_avg_sq"]))
        # the header's order: dW_l1, db1, dW_r1, dW_l0, db0, dW_r0
        order = [slots[i] for i in (3, 4, 5, 0, 1, 2)]
        P = (ctypes.c_void_p * 6)(*[o[0].data_ptr() for o in order])
        M = (ctypes.c_void_p * 6)(*[o[1].data_ptr() for o in order])
        V = (ctypes.c_void_p * 6)(*[o[2].data_ptr() for o in order])
        self._keep = step
        self.struct = _lib.AdamFold(P, M, V, step.data_ptr(), float(group["lr"]),
                                    float(b1), float(b2), float(group["eps"]), float(group["weight_decay"]))
        self.used = False

    @staticmethod
    def make(opt, model):
        """The spec when `opt` is ngnn.optim.Adam over exactly the two-layer
        stack's parameters (SAGE: six; SimpleGCN: four, W and b per conv) in
        fp32 with its state made (after a warm-up step), else None."""
        from .optim import Adam
        convs = getattr(model, "convs", None)
        if not isinstance(opt, Adam) or convs is None or len(convs) != 2 or len(opt.param_groups) != 1:
            return None
        params = []
        for c in convs:
            if hasattr(c, "lin_l") and getattr(c, "lin_r", None) is not None:
                params += [c.lin_l.weight, c.lin_l.bias, c.lin_r.weight]
            elif hasattr(c, "lin") and not hasattr(c, "lin_l") and getattr(c, "bias", None) is not None:
                params += [c.lin.weight, c.bias, None]  # GCNConv(normalize=False)
            else:
                return None
        live = [q for q in params if q is not None]
        if len(live) not in (4, 6) or (len(live) == 4 and (params[2], params[5]) != (None, None)):
            return None
        group = opt.param_groups[0]["params"]
        if len(group) != len(live) or {id(q) for q in group} != {id(q) for q in live}:
            return None
        # (ngnn.optim.Adam skips a parameter with no gradient -- a frozen one;
        # the folded reduction would update all six: no fold then)
        if not all(q.requires_grad for q in live):
            return None
        for q in live:
            s = opt.state.get(q, {})
            if (q.dtype != torch.float32 or not q.is_contiguous() or "step" not in s
                    or s["exp_avg"].dtype != torch.float32):
                return None
        if len({opt.state[q]["step"].data_ptr() for q in live}) != 1:
            return None
        return AdamFoldSpec(opt, params)


def sage2_backward(dy, block: Block, reduce: str, acts, agg0, params, p_drop: float, r_ptr: int,
                   rn_ptr: int, views, g_pre=None, root_free: bool = False):
    """Every weight gradient of the two-layer stack (include/ngnn.h
    ngnn_sage2_bwd): [dW_l0, db0, dW_r0, dW_l1, db1, dW_r1] from dy (rows <
    *r_ptr) with the forward's h (rows < *rn_ptr) and layer-0 aggregate.
    views: the data-parallel bucket's gradient views (or Nones).  g_pre: the
    scatter of dy onto the source rows, already built (LossHead), or None."""
    lib = _lib.load()
    x, h = acts[0], acts[1]
    wl0, bl0, wr0, wl1, bl1, wr1 = params
    dev = dy.device
    N, K0 = x.shape[0], wl0.shape[1]
    F1 = wl1.shape[0]
    w1l, w1r = wl1.detach(), wr1.detach()
    if w1l.stride(1) != 1 or w1r.stride(0) != w1l.stride(0) or w1r.stride(1) != 1:
        w1l, w1r = w1l.contiguous(), w1r.contiguous()
    grads = [(g.view(q.shape) if g is not None else torch.empty_like(q))
             for g, q in zip(views, (wl0, bl0, wr0, wl1, bl1, wr1))]
    if root_free:  # (ABI 18: a SimpleGCN stack -- no x reads, no W_r gradients)
        grads[2] = grads[5] = None
    nrows = block.n_dst
    ws = reserve_sage2_bwd(dev, nrows, K0, F1)
    yscale = dropout_scale(p_drop) if p_drop > 0.0 else 1.0
    fold = _adam_fold
    if fold is not None and not (len(params) == 6 and all(
            a.data_ptr() == b.data_ptr() for a, b in zip(params, fold.params))):
        fold = None
    if fold is not None:
        fold.used = True
    with _timing.span("sage2_bwd", 0, 0):
        rc = lib.ngnn_sage2_bwd(
            _lib.ptr(dy), dy.stride(0), F1, _lib.ptr(w1l), _lib.ptr(w1r), w1l.stride(0), _lib.ptr(h),
            h.stride(0), yscale, None if root_free else _lib.ptr(x), None if root_free else _lib.ptr(block.x_dev),
            None, None if root_free else _lib.ptr(block.xrow_dev),
            block.x_rows, x.stride(0), K0, _lib.ptr(agg0), agg0.stride(0), _lib.ptr(block.rowptr),
            _lib.ptr(block.col), nrows, r_ptr, rn_ptr, _lib.REDUCE[reduce], *(_lib.ptr(g) for g in grads[3:]),
            *(_lib.ptr(g) for g in grads[:3]), _lib.ptr(g_pre),
            None if fold is None else ctypes.byref(fold.struct), _lib.ptr(ws), ws.numel(),
            _lib.stream_handle(dev))
    _lib.check(rc, "ngnn_sage2_bwd")
    return grads


class _SAGEStack(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, block: Block, reduce: str, p_drop: float, seed: int, seed_dev, gouts,
                w_bf16: bool, head, *params):
        L = len(params) // 3
        acts, aggs = [x], []
        h = x
        ctx.h_partial = False
        ctx.sage2 = False
        p6 = sage2_params(params) if L == 2 else None
        if p6 is not None and sage2_ok(x, block, reduce, p6, w_bf16):
            ctx.sage2 = True
            h1, h, agg0, ctx.h_partial = sage2_forward(x, block, reduce, p6, p_drop, seed, seed_dev,
                                                       head=head, root0=params[2] is not None)
            if head is not None:
                h._ngnn_head = head  # (seed_cross_entropy takes the loss from it)
            acts += [h1, h]
            aggs += [agg0, None]
            L = 0  # (the per-layer loop below is skipped)
        for i in range(L):
            wl, bl, wr = params[3 * i:3 * i + 3]
            last = i == L - 1
            relu, p_i, seed_i = not last, (0.0 if last else p_drop), seed + 7919 * i
            x_dev = block.x_dev if i == 0 else None
            xrow = dict(xrow_dev=block.xrow_dev, x_rows=block.x_rows) if i == 0 else {}
            pk = block.wl_prepacked
            if (pk is not None and i == 0 and wr is not None and (len(pk) < 3 or pk[2].armed)
                    and pk[0].data_ptr() == wl.data_ptr() and pk[0].shape == wl.shape):
                xrow["wl_packed"] = pk[1]
                if len(pk) > 2:
                    pk[2].armed = False  # one forward per load (graphs.PackState)
            if wr is None and h.size(1) > wl.shape[0]:
                # GCN layer narrowing its input: transform first (PyG's order),
                # no saved aggregate (rebuilt for the rows backward needs)
                agg = None
                h = gcn_transform_first(h, block, wl, bl, relu, p_i, seed_i, seed_dev, x_dev,
                                        span=f"gcn_fwd_l{i}", **xrow)
            else:
                # the output layer aggregates in the F_out-wide space when it can
                # (its K-wide aggregate is rebuilt for the seed rows in backward)
                narrow = (wr is not None and last and i > 0
                          and narrow_ok(reduce, h.size(1), wl.shape[0], False, 0.0))
                agg = None if narrow else agg_buffer(h.size(0), h.size(1), h.device, wl.shape[0])
                # a bf16 model's hidden activations are bf16 rows (as the
                # reference's bf16 layers produce them): half the bytes written
                # here and read by the next layer and the backward.  (MAX keeps
                # fp32: its backward tie test reads the layer input; GCN stacks
                # keep fp32 too: their transform-first layers read fp32 rows.)
                h = sage_layer_fwd(h, block, reduce, wl, bl, wr, relu=relu, p_drop=p_i,
                                   seed=seed_i, agg_out=agg, seed_dev=seed_dev, x_dev=x_dev,
                                   span=f"sage_fwd_l{i}", narrow=narrow, w_bf16=w_bf16,
                                   out_bf16=(w_bf16 and not last and reduce != "max"
                                             and wr is not None), **xrow)
            acts.append(h)
            aggs.append(agg)
        if _debug_acts is not None:
            _debug_acts.append([a.detach().float().clone() for a in acts[1:-1]])
        ctx.block, ctx.reduce, ctx.p_drop, ctx.L = block, reduce, p_drop, len(params) // 3
        ctx.gouts = gouts  # _GradViews (buffers the weight gradients go into) or None
        ctx.save_for_backward(*acts, *aggs, *params)
        return h

    @staticmethod
    def backward(ctx, dout):
        block, reduce, p, L = ctx.block, ctx.reduce, ctx.p_drop, ctx.L
        saved = ctx.saved_tensors
        acts, aggs, params = saved[:L + 1], saved[L + 1:2 * L + 1], saved[2 * L + 1:]
        lib = _lib.load()
        dev = dout.device
        stream = _lib.stream_handle(dev)
        need_dx = ctx.needs_input_grad[0]
        if need_dx and block.x_dev is not None:
            raise _lib.NGNNError("input gradient of a zero-copy slot input is not supported")
        N = block.n_dst
        grads = [None] * (3 * L)
        # the claimed bucket views serve the FIRST backward only (a second one,
        # retain_graph, would write into a view autograd already adopted)
        gv = ctx.gouts
        views = gv.views if (gv is not None and gv.live) else [None] * (3 * L)
        if gv is not None:
            gv.live = False
        dy = dout if dout.stride(1) == 1 else dout.contiguous()
        # bnd[L] = rows of dout that can be nonzero; bnd[i] = same for d(acts[i])
        # (prefix_stats takes max(bnd[i], R, ...), so R is a valid initial bnd[i])
        rows_hint = getattr(dout, "_ngnn_nonzero_rows", None)  # set by ngnn.losses
        # the producer's precomputed top-layer bound (graph slot): no prefix-stats launch
        pre_top = (L > 0 and block.r_next is not None and rows_hint is not None
                   and int(rows_hint) == block.r_next[1])
        # bound entries some launch below writes: row_extent (bnd[L]) without a
        # hint, prefix stats for layers L-1 .. 1 (and 0 when dx is needed)
        written = rows_hint is None or any(
            not (pre_top and i == L - 1) for i in range(L - 1, -1 if need_dx else 0, -1))
        if written:
            # a fresh copy of the cached constant (a device-to-device memcpy:
            # no fill kernel in the step)
            bnd = torch.empty(L + 1, dtype=torch.int32, device=dev)
            bnd.copy_(const_bounds(dev, L, int(rows_hint) if rows_hint is not None else 0))
        else:  # read-only: a cached constant (no fill launch per step)
            bnd = const_bounds(dev, L, int(rows_hint))
        bp = [bnd.data_ptr() + 4 * j for j in range(L + 1)]
        if ctx.h_partial and not pre_top:
            # the forward wrote h only below the slot's R' (sage2_forward)
            raise _lib.NGNNError("this backward needs hidden rows past the slot's bound: the loss "
                                 "must read rows < the slot's batch size (seed_cross_entropy)")
        if pre_top:
            bp[L - 1] = block.r_next[0].data_ptr()
        bptr = lambda j: bp[j]  # noqa: E731
        if (ctx.sage2 and pre_top and not need_dx and _use_bwd2
                and not torch.are_deterministic_algorithms_enabled()):
            # (a loss head's gradient arrives with its scatter done: g_pre)
            return (None, None, None, None, None, None, None, None, None,
                    *_absent_none(params, sage2_backward(dy, block, reduce, acts, aggs[0], sage2_params(params),
                                                         p, bptr(2), bptr(1), views,
                                                         g_pre=getattr(dout, "_ngnn_g_pre", None),
                                                         root_free=params[2] is None)))
        if (ctx.sage2 and not ctx.h_partial and not need_dx and _use_bwd2
                and not torch.are_deterministic_algorithms_enabled()):
            # an eager step (the reference loop after the Option-B swap: no
            # graph slot, F.cross_entropy on out[:batch_size]): the same
            # two-layer backward, its row bounds from dout on the device --
            # R = the rows of dout that can be nonzero, R' their sources'
            # bound -- instead of the per-layer kernels (which rebuilt layer
            # 1's aggregate over every row without a loss hint)
            if rows_hint is None:
                _lib.check(lib.ngnn_row_extent(_lib.ptr(dy), dy.stride(0), N, dy.size(1), bptr(L),
                                               stream), "ngnn_row_extent")
            _lib.check(lib.ngnn_block_prefix_stats(_lib.ptr(block.rowptr), _lib.ptr(block.col),
                                                   bptr(L), None, bptr(L - 1), block.E, stream),
                       "ngnn_block_prefix_stats")
            return (None, None, None, None, None, None, None, None, None,
                    *_absent_none(params, sage2_backward(dy, block, reduce, acts, aggs[0], sage2_params(params),
                                                         p, bptr(2), bptr(1), views, root_free=params[2] is None)))
        if rows_hint is None:
            _lib.check(lib.ngnn_row_extent(_lib.ptr(dy), dy.stride(0), N, dy.size(1), bptr(L),
                                           stream), "ngnn_row_extent")
        # input-gradient scatter: float atomics by default (as the reference's CUDA
        # index_add_); the source-grouped CSR gather when determinism is requested
        deterministic = torch.are_deterministic_algorithms_enabled()
        t = block.transposed() if (deterministic and (L > 1 or need_dx)) else None
        red = _lib.REDUCE[reduce]
        for i in reversed(range(L)):
            h_in, y_out, agg = acts[i], acts[i + 1], aggs[i]
            if _debug_grads is not None:  # test/debug hook: d(acts[i+1]) per layer
                _debug_grads.append((i, dy.detach().clone(),
                                     None if agg is None else agg.detach().clone(),
                                     h_in.detach().clone()))
            wl, bl, wr = params[3 * i:3 * i + 3]
            gcn = wr is None  # GCN layer: SAGE with W_r = 0 (no root-term gradient)
            if gcn:
                wr = _zeros_like_cached(wl)
            Fo, K = wl.shape
            hidden = i != L - 1
            ymask = y_out if hidden else None
            y_bf16 = ymask is not None and ymask.dtype == torch.bfloat16
            yscale = dropout_scale(p) if (hidden and p > 0.0) else 1.0
            # gradient buffers: the data-parallel bucket's views when the caller
            # registered them (a fresh view each time, so autograd adopts it as
            # .grad instead of copying it), else new tensors
            dwl, dbl, dwr = (
                (g.view(q.shape) if g is not None else torch.empty_like(q))
                for g, q in zip(views[3 * i:3 * i + 3], (wl, bl, wr)))
            if gcn:
                dwr = _workspace(dev, "gcn_dwr", wr.numel() * 4).view(torch.float32)[
                    :wr.numel()].view(wr.shape)
            if agg is None:
                if i == 0 and block.x_dev is not None:  # (zero_copy_ok excludes it)
                    raise _lib.NGNNError("layer-0 aggregate rebuild from a zero-copy input")
                # narrow-mode layer: the K-wide aggregate the weight gradient
                # reads (rows < R) gathered now -- R rows when the loss told us
                # R (the seed rows), else every row
                R = int(rows_hint) if (rows_hint is not None and i == L - 1) else N
                agg = torch.empty(max(R, 1), K, dtype=torch.float32, device=dev)
                with _timing.span("sage_agg_seed_rows", 0, 0):
                    _lib.check(lib.ngnn_seg_agg_fwd(
                        _lib.ptr(h_in), h_in.stride(0), K, _lib.ptr(block.rowptr),
                        _lib.ptr(block.col), R, red,
                        _lib.BF16 if h_in.dtype == torch.bfloat16 else _lib.F32, _lib.ptr(agg),
                        agg.stride(0), stream), "ngnn_seg_agg_fwd")
            wsb = lib.ngnn_sage_wgrad_workspace_bytes(Fo, K)
            ws = _workspace(dev, "wgrad", wsb)
            with _timing.span("sage_wgrad", 0, 0):  # row bound is device-side: no host count
                rc = lib.ngnn_sage_wgrad(
                    _lib.ptr(dy), dy.stride(0), _lib.ptr(ymask),
                    ymask.stride(0) if ymask is not None else Fo, yscale, _lib.ptr(h_in),
                    _lib.ptr(block.x_dev) if i == 0 else None,
                    None, _lib.ptr(block.xrow_dev) if i == 0 else None,
                    block.x_rows if i == 0 else 0,
                    int(h_in.dtype == torch.bfloat16) | (2 if y_bf16 else 0), h_in.stride(0),
                    _lib.ptr(agg), agg.stride(0), _lib.ptr(block.rowptr), N,
                    bptr(i + 1), Fo, K, _lib.ptr(dwl), _lib.ptr(dbl), _lib.ptr(dwr),
                    _lib.ptr(ws), ws.numel(), stream)
            _lib.check(rc, "ngnn_sage_wgrad")
            grads[3 * i:3 * i + 3] = [dwl, dbl, None if gcn else dwr]
            if i == 0 and not need_dx:
                break
            if not (pre_top and i == L - 1):
                _lib.check(lib.ngnn_block_prefix_stats(_lib.ptr(block.rowptr), _lib.ptr(block.col),
                                                       bptr(i + 1), None, bptr(i), block.E, stream),
                           "ngnn_block_prefix_stats")
            if y_bf16:
                # the input-gradient kernels read an fp32 mask: widen its rows
                # below the output-gradient bound (device-side)
                ym = _workspace(dev, "ymask_f32", N * Fo * 4).view(torch.float32)[:N * Fo].view(N, Fo)
                _lib.check(lib.ngnn_widen_bf16_rows(_lib.ptr(ymask), ymask.stride(0), Fo, N,
                                                    bptr(i + 1), _lib.ptr(ym), Fo, stream),
                           "ngnn_widen_bf16_rows")
                ymask = ym
            if not deterministic and Fo < K and reduce in ("sum", "mean"):
                # narrow-space path: scatter dz (Fo wide), then one MFMA pass
                dh = torch.empty(N, K, dtype=torch.float32, device=dev)
                wlc, wrc = wl.detach().contiguous(), wr.detach().contiguous()
                gws = _workspace(dev, ("dgrad_lowdim", Fo, K),  # g stays zero per shape
                                 lib.ngnn_sage_dgrad_lowdim_workspace_bytes(N, Fo, K), zero=True)
                with _timing.span("sage_dgrad_lowdim", 0, 0):
                    rc = lib.ngnn_sage_dgrad_lowdim(
                        _lib.ptr(dy), dy.stride(0), _lib.ptr(ymask),
                        ymask.stride(0) if ymask is not None else Fo, yscale, _lib.ptr(wlc),
                        _lib.ptr(wrc), wlc.stride(0), Fo, K, _lib.ptr(block.rowptr),
                        _lib.ptr(block.col), N, bptr(i + 1), bptr(i), red, _lib.ptr(dh),
                        dh.stride(0), int(i == 0), _lib.ptr(gws), gws.numel(), stream)
                if rc == _lib.OK:
                    dy = dh
                    continue
                if rc != _lib.E_SHAPE:
                    _lib.check(rc, "ngnn_sage_dgrad_lowdim")
            if not deterministic and _dgrad_fused_ok(Fo, K):
                # atomic path: per-row VALU products + scatter, no dgrad GEMM launch
                dh = torch.empty(N, K, dtype=torch.float32, device=dev)
                wlc, wrc = wl.detach().contiguous(), wr.detach().contiguous()
                with _timing.span("sage_dgrad_fused", 0, 0):
                    rc = lib.ngnn_sage_dgrad_fused(
                        _lib.ptr(dy), dy.stride(0), _lib.ptr(ymask),
                        ymask.stride(0) if ymask is not None else Fo, yscale, _lib.ptr(wlc),
                        _lib.ptr(wrc), Fo, K, _lib.ptr(block.rowptr), _lib.ptr(block.col), N,
                        bptr(i + 1), bptr(i), red, _lib.ptr(h_in), h_in.stride(0), _lib.ptr(agg),
                        agg.stride(0), _lib.ptr(dh), dh.stride(0), int(i == 0), stream)
                _lib.check(rc, "ngnn_sage_dgrad_fused")
                dy = dh
                continue
            # dgrad GEMM: [dz W_l | dz W_r] on rows < R (ReLU/dropout backward in the staging)
            pk = pack_dgrad_weight(wl, wr)
            dg = torch.empty(N, 2 * K, dtype=torch.float32, device=dev)
            with _timing.span("sage_dgrad", 0, 0):
                _gemm_layer(dy, Fo, N, None, "mean", None, pk, None, 2 * K, dg, False, 0.0, 0,
                            n_rows_dev=bptr(i + 1), xmask=ymask, xscale=yscale)
            dh = torch.empty(N, K, dtype=torch.float32, device=dev)
            if deterministic:
                gws = _workspace(dev, "dgrad", lib.ngnn_sage_dgrad_workspace_bytes(N, K, red))
                with _timing.span("sage_dgrad_gather", 0, 0):
                    rc = lib.ngnn_sage_dgrad_gather(
                        _lib.ptr(dg), 2 * K, _lib.ptr(dg) + 4 * K, 2 * K, _lib.ptr(block.rowptr),
                        _lib.ptr(block.col), _lib.ptr(t.rowptr), _lib.ptr(t.col), N, bptr(i + 1),
                        bptr(i), K, red, _lib.ptr(h_in), h_in.stride(0), _lib.ptr(agg),
                        agg.stride(0), _lib.ptr(dh), dh.stride(0), int(i == 0), _lib.ptr(gws),
                        gws.numel(), stream)
                _lib.check(rc, "ngnn_sage_dgrad_gather")
            else:
                with _timing.span("sage_dgrad_scatter", 0, 0):
                    rc = lib.ngnn_sage_dgrad_scatter(
                        _lib.ptr(dg), 2 * K, _lib.ptr(dg) + 4 * K, 2 * K, _lib.ptr(block.rowptr),
                        _lib.ptr(block.col), N, bptr(i + 1), bptr(i), K, red, _lib.ptr(h_in),
                        h_in.stride(0), _lib.ptr(agg), agg.stride(0), _lib.ptr(dh), dh.stride(0),
                        int(i == 0), stream)
                _lib.check(rc, "ngnn_sage_dgrad_scatter")
            dy = dh
        dx = dy if (need_dx and L > 0) else None
        return (dx, None, None, None, None, None, None, None, None, *grads)


_IO_DTYPES = (torch.float32, torch.bfloat16)


def sage_stack_supported(model, x) -> bool:
    if not x.is_cuda or x.dtype not in _IO_DTYPES or x.dim() != 2:
        return False
    if getattr(model, "use_bn", False):
        return False
    convs = model.convs
    aggr = convs[0].aggr
    for conv in convs:
        # (the convs' own parameter dicts: model.parameters() walks the module
        # tree, ~10 us of the host-bound eager step)
        if conv.aggr != aggr:
            return False
        for m in (conv.lin_l, getattr(conv, "lin_r", None)):
            for p in (() if m is None else m._parameters.values()):
                if p is not None and p.dtype not in _IO_DTYPES:
                    return False
    return True


class _ConvCall:
    """A single conv run as a one-layer stack: no dropout (the reference
    wrapper applies relu / F.dropout itself, sage.py:35-38)."""
    dropout = 0.0
    training = False


def conv_supported(conv, x) -> bool:
    return (x.is_cuda and x.dtype in _IO_DTYPES and x.dim() == 2
            and all(p.dtype in _IO_DTYPES for p in conv.parameters()))


def sage_conv(conv, x, block: Block) -> torch.Tensor:
    """SAGEConv.forward (PyG 2.5.1 semantics, sage.py:34) as a one-layer fused
    stack: forward on the row-tile kernel (aggregate saved), backward =
    weight gradient + input gradient kernels; the input gradient covers every
    row (the wrapper's relu / dropout backward reads all of it)."""
    aggr = "sum" if conv.aggr == "add" else conv.aggr
    params = [conv.lin_l.weight, conv.lin_l.bias, conv.lin_r.weight]
    return _run_stack(_ConvCall, x, block, 0, None, params, aggr, keep_bf16_x=True)


def gcn_conv(conv, x, block: Block) -> torch.Tensor:
    """GCNConv(normalize=False).forward (convolution.py:31) as a one-layer
    fused GCN stack (W_r = 0, sum aggregation)."""
    return _run_stack(_ConvCall, x, block, 0, None, [conv.lin.weight, conv.bias, None], "sum")


def zero_copy_ok(model, n_rows: int, in_dim: int, table_rows: int = 0) -> bool:
    """Can a HIP-graph slot hand this model's layer 0 the batch's feature rows
    in place (ngnn_sage_fwd_raw's x_dev)?  Only the fused SAGE stack reads
    x_dev, and only the row-tile kernel accepts it: K % 4 == 0 and 32-bit
    buffer offsets over the slot's rows (x, the output, the saved aggregate).
    table_rows > 0: the rows are gathered from a feature table of that many
    rows (fused x[n_id]; the weight gradient then needs it under 2 GiB)."""
    # only this package's fused stacks read the slot's x through x_dev; any
    # other model (e.g. a reference wrapper around ngnn convs) reads the slot
    from .models import SAGE, SimpleGCN
    if not isinstance(model, (SAGE, SimpleGCN)):
        return False
    if not isinstance(getattr(model, "convs", None), torch.nn.ModuleList):
        return False
    if getattr(model, "use_bn", False):
        return False
    c0 = model.convs[0]
    wide = False
    if hasattr(c0, "lin_r"):
        if len({c.aggr for c in model.convs}) != 1:
            return False
        fo = c0.lin_r.weight.shape[0]
        # layer 0 on the wide path (Amazon-Computers' 767 -> 512): its
        # kernels read the rows in place at 4-B alignment, any K
        wide = (not table_rows and c0.lin_r.weight.dtype == torch.float32
                and bool(_lib.load().ngnn_sage_wide_preferred(in_dim, fo, int(_exact_f32))))
    elif hasattr(c0, "lin"):  # SimpleGCN
        fo = c0.lin.weight.shape[0]
        if in_dim > fo:  # transform-first layer 0: backward rebuilds its aggregate from x
            return False
    else:
        return False
    # the layer-0 gather reads x through one 32-bit-offset resource (< 3.75
    # GiB, ngnn_sage_rt.hip kRangeMax); outputs are addressed per tile
    lim = 0xF0000000 - 4096
    if table_rows and table_rows * in_dim * 4 >= 2**31:
        return False
    if wide:
        return n_rows * in_dim * 4 <= lim
    return (in_dim % 4 == 0 and max(n_rows, table_rows) * in_dim * 4 <= lim
            and -(-in_dim // 16) <= 79)


def gcn_stack_supported(model, x) -> bool:
    return (x.is_cuda and x.dtype in _IO_DTYPES and x.dim() == 2
            and all(p.dtype in _IO_DTYPES for p in model.parameters()))


def gcn_stack(model, x, block: Block, seed: int, seed_dev=None) -> torch.Tensor:
    """SimpleGCN's forward (convolution.py:29-35) as ONE autograd node on the
    fused kernels: each GCNConv(normalize=False) is the SAGE layer with W_r
    = 0 and a sum aggregation (aggregate-first when F_in <= F_out, PyG's
    transform-first otherwise), the backward the bounded SAGE backward.
    bf16 models: bf16 storage, fp32 arithmetic (as sage_stack)."""
    params = []
    for conv in model.convs:
        params += [conv.lin.weight, conv.bias, None]
    return _run_stack(model, x, block, seed, seed_dev, params, "sum")


def sage_stack(model, x, block: Block, seed: int, seed_dev=None) -> torch.Tensor:
    """bf16 models (config #3 of BASELINE.json) run with bf16 storage at the
    module boundary: inputs and parameters are widened to fp32 for the fused
    fp32 kernels (autograd narrows the gradients back) and the logits are
    returned in x's dtype -- fp32 arithmetic inside, no bf16 MFMA path."""
    params = []
    for conv in model.convs:
        params += [conv.lin_l.weight, conv.lin_l.bias, conv.lin_r.weight]
    aggr = "sum" if model.convs[0].aggr == "add" else model.convs[0].aggr
    return _run_stack(model, x, block, seed, seed_dev, params, aggr, keep_bf16_x=True)


class _GradViews:
    """The bucket views (ngnn.distributed.GradAllReduce) one pending stack
    node may write its weight gradients into.  A parameter's view goes to ONE
    node at a time: the node claims it at forward time and gives it up in its
    first backward (or when its graph is freed without one -- the parameter
    holds only a weak reference).  Without the claim, two forwards before one
    backward (the reference's pipeline_contrast.py:146-154 runs the model on
    several batches per step) would both write into the same view, autograd
    would adopt the first write and then add the view to itself: 2 g2 instead
    of g1 + g2."""

    __slots__ = ("views", "live", "__weakref__")

    def __init__(self, n: int):
        self.views = [None] * n
        self.live = True


_grad_views_seen = False  # set once any parameter got a bucket view


def note_grad_views() -> None:
    """ngnn.distributed.GradAllReduce registered a bucket view (until then the
    eager step skips the per-parameter claim scan)."""
    global _grad_views_seen
    _grad_views_seen = True


def _claim_grad_views(params) -> "_GradViews | None":
    """Views for the fp32 parameters whose .grad is unset (autograd will adopt
    them) and whose view no other pending node holds; None when there are none."""
    if not _grad_views_seen or not torch.is_grad_enabled():
        return None
    gv = _GradViews(len(params))
    for i, q in enumerate(params):
        if (q is None or q.grad is not None or q.dtype != torch.float32
                or not q.requires_grad):
            continue
        v = getattr(q, "_ngnn_grad_out", None)
        if v is None:
            continue
        held = getattr(q, "_ngnn_grad_claim", None)
        holder = held() if held is not None else None
        if holder is not None and holder.live:
            continue  # another forward's backward is still to write it
        q._ngnn_grad_claim = weakref.ref(gv)
        gv.views[i] = v
    return gv if any(v is not None for v in gv.views) else None


_use_eager_ext = True  # (tests flip it to compare the C++ node with _SAGEStack)
eager_ext_calls = 0  # (counted: the tests check which node ran)


def _eager_sage2(x, block: Block, reduce: str, p_drop: float, seed: int, params):
    """The eager two-layer SAGE stack through the C++ autograd node
    (csrc/ngnn_eager.cpp: the launches _SAGEStack makes on this path --
    sage2_forward with every row of h kept; row extent, prefix stats and
    sage2_backward -- with ~100 us less host time per step), or None when
    the call is not that path: a graph slot's block (device counts, fused
    x[n_id], bounds, loss head, prepacked weights), bucket gradient views,
    an input gradient, a GCN stack, deterministic mode, the bench's per-launch
    timer, the debug hooks, or the module not built."""
    if (not _use_eager_ext or len(params) != 6 or _debug_acts is not None or _debug_grads is not None
            or not _use_bwd2 or _adam_fold is not None or x.requires_grad or _timing.timing()
            or torch.are_deterministic_algorithms_enabled()):
        return None
    if (block.x_dev is not None or block.xrow_dev is not None or block.n_rows_dev is not None
            or block.n_edge_rows_dev is not None or block.r_next is not None or block.wl_prepacked is not None
            or block.n_active is None or x.size(0) != block.n_dst):
        return None
    if any(q is None or not q.is_contiguous() for q in params) or not sage2_ok(x, block, reduce, params, False):
        return None
    # agg0 [N, K0] unpadded (agg_buffer pads K0 % 4 != 0 rows)
    if x.size(1) % 4:
        return None
    ext = _eager.load()
    if ext is None:
        return None
    global eager_ext_calls
    eager_ext_calls += 1
    N, K0 = x.shape
    F1 = params[3].shape[0]
    dev = x.device
    ws_f = _workspace(dev, "sage2", _ws_size("ngnn_sage2_workspace_bytes", K0, F1, N))
    ws_b = reserve_sage2_bwd(dev, block.n_dst, K0, F1)
    yscale = dropout_scale(p_drop) if p_drop > 0.0 else 1.0
    n_edge = min(int(block.n_active), N)
    return ext.sage2(x, *params, block.rowptr, block.col, n_edge, block.E, _lib.REDUCE[reduce], p_drop, yscale,
                     _i64_bits(seed), ws_f, ws_b, _lib.stream_handle(dev))


def _i64_bits(v: int) -> int:
    """The uint64 bits of v (the C ABI's seed) as the int64 pybind takes."""
    v &= 2**64 - 1
    return v - 2**64 if v >= 2**63 else v


def _run_stack(model, x, block: Block, seed: int, seed_dev, params, aggr: str,
               keep_bf16_x: bool = False) -> torch.Tensor:
    out_dtype = x.dtype
    # weight gradients straight into registered bucket views (ngnn.distributed.GradAllReduce)
    # when autograd will adopt them (see _GradViews)
    gouts = None
    # a bf16 model's weights are bf16-exact once widened: one-part split images
    w_bf16 = all(q is None or q.dtype == torch.bfloat16 for q in params)
    if out_dtype != torch.float32 or any(q is not None and q.dtype != torch.float32 for q in params):
        # bf16 features stay bf16 for a SAGE stack's layer 0 (the kernels read
        # bf16 rows, NGNN_X_BF16: half the bytes, no widened copy) unless an
        # input gradient is wanted; everything else is widened
        if not (keep_bf16_x and x.dtype == torch.bfloat16 and not x.requires_grad
                and bf16_rows_ok(x)):
            x = x.float()
        params = widen_params(params)
    else:
        gouts = _claim_grad_views(params)
    p = model.dropout if model.training else 0.0
    xc = x if (x.stride(1) == 1 and x.stride(0) >= x.size(1)) else x.contiguous()
    head = block.loss_head.start() if (out_dtype == torch.float32 and head_ok(block, xc, params)) else None
    out = None
    if head is None and gouts is None and seed_dev is None and out_dtype == torch.float32:
        out = _eager_sage2(xc, block, aggr, float(p), int(seed), params)
    if out is None:
        out = _SAGEStack.apply(xc, block, aggr, float(p), int(seed), seed_dev, gouts, w_bf16, head,
                               *params)
    if out_dtype == torch.float32:
        return out
    if out_dtype == torch.bfloat16 and out.is_contiguous() and out.dim() == 2:
        # a graph slot whose loss reads rows < B only (block.r_next[2]): the
        # bf16 logits of those rows alone (the other rows' fp32 logits stay
        # on the output as _ngnn_f32) -- the cast of a 1.5 M-row block's
        # logits was 69 us of the 3-layer products step
        rn = block.r_next
        rows = rn[1] if (rn is not None and len(rn) > 2 and rn[2]) else out.size(0)
        y = _StackOutBF16.apply(out, block.n_rows_dev, rows)
        if rows < out.size(0):
            y._ngnn_f32 = out.detach()
        return y
    from .losses import cast_keep_rows
    return cast_keep_rows(out, out_dtype)


def _cast_tensors(src, dst, to_bf16: bool) -> None:
    import ctypes
    n = len(src)
    for i in range(0, n, 16):  # (16 tensors per launch)
        a, b = src[i:i + 16], dst[i:i + 16]
        k = len(a)
        S = (ctypes.c_void_p * k)(*[t.data_ptr() for t in a])
        D = (ctypes.c_void_p * k)(*[t.data_ptr() for t in b])
        N = (ctypes.c_int64 * k)(*[t.numel() for t in a])
        _lib.check(_lib.load().ngnn_cast_tensors(k, S, D, N, int(to_bf16), _lib.stream_handle(a[0].device)),
                   "ngnn_cast_tensors")


class _WidenParams(torch.autograd.Function):
    """A bf16 model's parameters as fp32 tensors for the fused kernels:
    ONE ngnn_cast_tensors launch forward (bf16 -> fp32, exact) and one
    backward (the fp32 gradients rounded to the parameters' bf16) --
    Tensor.float() and its autograd backward were an ATen copy kernel per
    tensor and direction (~18 per step of the products 3-layer bf16 model)."""

    @staticmethod
    def forward(ctx, *params):
        outs = [torch.empty(q.shape, dtype=torch.float32, device=q.device) for q in params]
        _cast_tensors([q.contiguous() for q in params], outs, to_bf16=False)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        live = [i for i, g in enumerate(grads) if g is not None]
        outs = [None] * len(grads)
        if live:
            src = [grads[i].contiguous() for i in live]
            dst = [torch.empty(g.shape, dtype=torch.bfloat16, device=g.device) for g in src]
            _cast_tensors(src, dst, to_bf16=True)
            for i, d in zip(live, dst):
                outs[i] = d
        return tuple(outs)


def widen_params(params):
    """fp32 views of the stack's parameters: bf16 ones through _WidenParams
    (one launch each way), fp32 ones as they are, None kept."""
    idx = [i for i, q in enumerate(params) if q is not None and q.dtype == torch.bfloat16]
    out = [None if (q is None or q.dtype == torch.bfloat16) else q.float() for q in params]
    if idx:
        wide = _WidenParams.apply(*[params[i] for i in idx])
        if not isinstance(wide, tuple):
            wide = (wide,)
        for i, w in zip(idx, wide):
            out[i] = w
    return out


_out_grads: dict = {}


class _StackOutBF16(torch.autograd.Function):
    """The stack's fp32 logits handed back in bf16 (a bf16 model's output
    dtype) by one ngnn_cast_f32_bf16 launch.  Backward: the only consumer of
    its gradient is _SAGEStack.backward, which reads rows < R of dout when the
    loss says R (ngnn.losses' row hint) -- so only those rows are widened,
    into a cached buffer, and the hint travels on."""

    @staticmethod
    def forward(ctx, x, rows_dev=None, rows=None):
        # (rows_dev: a graph slot's device row count -- only the block's real
        # rows are cast; the slot's padding rows of y are left unwritten;
        # rows: a host cap, the rows a graph slot's loss reads)
        y = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
        n = x.size(0) if rows is None else min(int(rows), x.size(0))
        _lib.check(_lib.load().ngnn_cast_f32_bf16_rows(_lib.ptr(x), _lib.ptr(y), n, x.size(1),
                                                       _lib.ptr(rows_dev), _lib.stream_handle(x.device)),
                   "ngnn_cast_f32_bf16_rows")
        return y

    @staticmethod
    def backward(ctx, g):
        rows = getattr(g, "_ngnn_nonzero_rows", None)
        if rows is None:
            return g.float(), None, None
        key = (g.device, tuple(g.shape))
        buf = _out_grads.get(key)
        if buf is None:
            buf = torch.empty(g.shape, dtype=torch.float32, device=g.device)
            _out_grads[key] = buf
        R = min(int(rows), g.size(0))
        if g.dtype == torch.bfloat16 and g.dim() == 2 and g.stride(1) == 1:
            _lib.check(_lib.load().ngnn_widen_bf16_rows(_lib.ptr(g), g.stride(0), g.size(1), R, None,
                                                        _lib.ptr(buf), buf.stride(0),
                                                        _lib.stream_handle(g.device)),
                       "ngnn_widen_bf16_rows")
        else:
            buf[:R].copy_(g[:R])
        buf._ngnn_nonzero_rows = R  # rows >= R are stale: the stack never reads them
        return buf, None, None
