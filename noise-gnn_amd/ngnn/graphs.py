"""HIP-graph replay of the training step (the reference's loop body,
pipeline.py:152-169: forward on a NeighborLoader block, loss on the seed rows,
backward, optimizer step) over static, padded input slots.

Every launch of the step -- CSR build, both fused layer kernels, loss,
backward kernels, Adam -- is captured once into a HIP graph (through
``torch.cuda.CUDAGraph``) and replayed per batch, so the host issues one
graph launch instead of ~30 kernel launches and ~100 Python/ATen calls.
The step is capturable because the ngnn path never reads device values on the
host: block row bounds, backward receptive-field bounds and the dropout seed
live on the device.  The slot load (one launch before each replay) also
writes the target-grouped CSR of the padded edges and advances the dropout
seed, so the graph holds no CSR-build or RNG launches.  Edges must be
target-sorted (NeighborLoader's order).

Shapes are static: the slot holds ``n_cap`` node rows and ``e_cap`` edges.
The feature rows are not copied for a replay: the slot load stores the
batch's address in a device word the captured layer-0 kernels read
(zero-copy), so the batch tensor must stay alive until the step completes
(the step keeps a reference until the next load).
A batch with N nodes and E edges fills rows ``[0, N)`` and edges ``[0, E)``;
the padding edges are self-loops spread evenly over the padding rows
``[N, n_cap)`` (targets stay non-decreasing, no row gets more than a few), so
padded rows never feed a real row and never receive gradient (the loss reads
rows < batch_size only).  A device scalar holds N; the forward kernels read it
and skip the padding rows, so a generous slot costs memory, not time.

The gradient all-reduce of seed-sharded data parallelism (RCCL) runs between
two graphs (forward+backward+bucket pack, then bucket unpack+optimizer step),
outside capture: one collective call per step on the host.
"""
from __future__ import annotations

import torch

from . import _lib
from .block import CSR, block_cache, hint_edge_index
from .loader import IndexedRows
from .losses import seed_cross_entropy


class GraphedTrainStep:
    def __init__(self, model, optimizer, batch_size: int, n_cap: int, e_cap: int, in_dim: int,
                 device, reducer=None, loss_fn=None, warmup: int = 3):
        if not optimizer.defaults.get("capturable", False):
            raise ValueError("GraphedTrainStep needs an optimizer built with capturable=True")
        self.model, self.opt, self.reducer = model, optimizer, reducer
        self.B, self.n_cap, self.e_cap = int(batch_size), int(n_cap), int(e_cap)
        # loss_fn(out, y, batch_size): default == F.cross_entropy(out[:B], y[:B])
        self.loss_fn = loss_fn or seed_cross_entropy
        self.warmup = warmup
        dev = torch.device(device)
        self.x = torch.zeros(self.n_cap, in_dim, dtype=torch.float32, device=dev)
        self.ei = torch.zeros(2, self.e_cap, dtype=torch.int64, device=dev)
        self.y = torch.zeros(self.B, dtype=torch.int64, device=dev)
        self.n_valid = torch.full((1,), self.n_cap, dtype=torch.int32, device=dev)
        # the slot load also writes the CSR of the padded edges and advances
        # the dropout seed, so the captured step builds neither
        self.rowptr = torch.zeros(self.n_cap + 1, dtype=torch.int32, device=dev)
        self.col = torch.zeros(self.e_cap, dtype=torch.int32, device=dev)
        self.seed_state = torch.randint(0, 2**62, (1,), dtype=torch.int64).to(dev)
        # zero-copy input: the slot load stores the batch's feature address
        # here and the captured layer-0 kernels read the rows in place
        self.x_dev = torch.zeros(1, dtype=torch.int64, device=dev)
        # input-gradient row bound of the top layer (prefix stats for R = B),
        # written by the slot load so the captured backward needs no bound launch
        # (int64 word: generation << 32 | bound; consumers read the low half)
        self.r_next = torch.zeros(1, dtype=torch.int64, device=dev)
        # rows past the batch's last target have no in-edges (dense forward kernel)
        self.n_edge_rows = torch.zeros(1, dtype=torch.int32, device=dev)
        # fused x[n_id]: when captured on an IndexedRows batch, x_dev holds the
        # feature table's address and this word the batch's n_id (0: plain
        # rows); x_rows = the table's rows the captured kernels range over
        self.xrow_dev = torch.zeros(1, dtype=torch.int64, device=dev)
        self.x_rows = 0
        self.col_x = None  # layer 0's gather columns (table rows), allocated at capture
        self._gen = 0
        self._x_live = None  # the loaded batch's features, kept alive until the next load
        self.g_fb = self.g_opt = None
        self.loss = None
        self.out = None
        self._split_reduce = False
        self._one = None
        self.zero_copy = True
        # (layer-0 W_l, its packed image): the slot load packs the weight's
        # current values, the captured forward reads them prepacked
        self._pack = None
        self._head = None  # fused.LossHead (made at capture)
        self.folded = False  # the captured backward took the Adam step (fused.AdamFoldSpec)
        # the slot kernel's contract check (include/ngnn.h NGNN_SLOT_*): a word
        # in pinned host memory the device ORs into -- read by the host with
        # no device sync (load() raises on a word set by an earlier batch;
        # check_inputs() syncs and raises for the batches so far)
        self._err = torch.zeros(1, dtype=torch.int32).pin_memory()
        # its device twin (ABI 20): (generation << 32 | bits) of the newest
        # contract-breaking load; a one-rank captured step reads it and leaves
        # the parameters and the step count untouched for such a block
        self._gate = torch.zeros(1, dtype=torch.int64, device=dev)

    # ---- slot filling (stream-ordered device copies; no host syncs)
    def load(self, x: torch.Tensor, edge_index: torch.Tensor, y: torch.Tensor,
             zero_copy: bool = False, batch_size: int | None = None) -> None:
        """zero_copy: store x's address for the captured kernels instead of
        copying its rows into the slot (replays); the copy serves eager use
        of the slot (warm-up, tests).  batch_size: the block's seed count
        (default: the captured B).  x may be an IndexedRows (a batch of
        NeighborLoader(gather_features=False)): zero-copy replays of a step
        captured on one pass the feature table and n_id (the layer-0 kernels
        gather the rows); otherwise its rows are gathered here.  A short block (an epoch's last batch when
        drop_last is off) gets ignore_index (-100) labels on rows
        [batch_size, B), so the captured loss -- F.cross_entropy(out[:B],
        y[:B]) with the default ignore_index -- is exactly the reference's
        F.cross_entropy(out[:batch_size], y[:batch_size]) (pipeline.py:155-158):
        mean over the real seeds, zero gradient on the other rows."""
        xrow = None
        # a sync-free NeighborLoader batch (ABI 19): capacity-sized buffers,
        # the block's row / edge counts on the device -- N and E below are
        # then their bounds, the slot kernel reads the counts itself
        cnt = getattr(edge_index, "_ngnn_counts", None)
        if isinstance(x, IndexedRows):
            t, idx = x.table, x.index
            if (zero_copy and self.x_rows and t.dtype == torch.float32 and t.stride(1) == 1
                    and t.stride(0) == self.x.stride(0) and t.data_ptr() % 16 == 0
                    and t.size(0) <= self.x_rows and idx.dtype == torch.int64
                    and idx.is_contiguous()):
                xrow = idx
                x = t
            else:
                x = x.materialize()
        N, E = (x.size(0) if xrow is None else xrow.numel()), edge_index.size(1)
        if N + 1 > self.n_cap or E > self.e_cap:
            raise ValueError(f"batch (N={N}, E={E}) exceeds the slot ({self.n_cap}, {self.e_cap})")
        bs = self.B if batch_size is None else int(batch_size)
        if not 0 < bs <= min(self.B, N):
            raise ValueError(f"batch_size {bs} outside (0, min(B={self.B}, N={N})]")
        if x.dtype != self.x.dtype:  # the slot's dtype (bf16 slots: bf16-reading kernels)
            x = x.to(self.x.dtype)
        if x.stride(1) != 1 or x.stride(0) != self.x.stride(0) or x.data_ptr() % 16:
            x = x.clone(memory_format=torch.contiguous_format)
        # a step captured for indexed rows: the word gets n_id's address or 0
        xrow_word = self.xrow_dev if (zero_copy and self.x_rows) else None
        # the slot kernel's CSR assumes non-decreasing targets and ids in
        # [0, N): the kernel checks every edge and sets the pinned error word
        # (no host read-back of the targets per step); a word set by an
        # earlier batch raises here
        self._raise_if_bad()
        if edge_index.stride(1) != 1:
            edge_index = edge_index.contiguous()
        y = y[:bs].contiguous()
        if bs < self.B:  # rows [bs, B) carry no loss (F.cross_entropy's ignore_index)
            y = torch.cat([y, y.new_full((self.B - bs,), -100)])
        # one launch: x rows, edges + padding self-loops, labels, device row count
        # (bf16 rows move as float32 pairs: the slot kernel copies 32-bit words)
        xw = x.view(torch.float32) if x.dtype == torch.bfloat16 else x
        sx = self.x.view(torch.float32) if self.x.dtype == torch.bfloat16 else self.x
        _lib.check(_lib.load().ngnn_slot_load(
            _lib.ptr(xw), xw.stride(0), N, xw.size(1), _lib.ptr(edge_index), edge_index.stride(0), E,
            _lib.ptr(y), y.numel(), _lib.ptr(sx), sx.stride(0), self.n_cap,
            # replays read only the slot's CSR (the int64 edge copy serves eager
            # use and the deterministic mode's transposed CSR)
            None if (zero_copy and not torch.are_deterministic_algorithms_enabled())
            else _lib.ptr(self.ei), self.e_cap, _lib.ptr(self.y), _lib.ptr(self.n_valid),
            _lib.ptr(self.rowptr), _lib.ptr(self.col), _lib.ptr(self.seed_state),
            _lib.ptr(self.x_dev) if zero_copy else None, _lib.ptr(self.r_next), self._next_gen(),
            _lib.ptr(self.n_edge_rows), _lib.ptr(xrow), _lib.ptr(xrow_word),
            _lib.ptr(self.col_x) if xrow_word is not None else None,
            # pack job: layer 0's W_l in fragment order for the captured forward
            *((_lib.ptr(self._pack[0]), self._pack[0].stride(0), self._pack[0].shape[0],
               self._pack[0].shape[1], _lib.ptr(self._pack[1])) if self._pack is not None
              else (None, 0, 0, 0, None)),
            self._err.data_ptr(), _lib.ptr(cnt), _lib.ptr(self._gate), _lib.stream_handle(self.x.device)),
            "ngnn_slot_load")
        self._x_live = (x, xrow) if zero_copy else None
        if self._pack is not None:  # this load packed the current W_l: one forward may use it
            self._pack[2].armed = True

    def _raise_if_bad(self) -> None:
        bad = int(self._err[0])
        if bad:
            self._err.zero_()
            what = []
            if bad & _lib.SLOT_UNSORTED:
                what.append("targets not sorted (NeighborLoader's order: sort edge_index by "
                            "edge_index[1], stable)")
            if bad & _lib.SLOT_RANGE:
                what.append("node ids outside [0, N)")
            raise ValueError("GraphedTrainStep: a batch loaded into the slot broke its contract -- "
                             + "; ".join(what) + " -- and was trained on a wrong CSR")

    def check_inputs(self) -> None:
        """Synchronize and raise if any batch loaded so far broke the slot's
        contract (load() reports such a batch at the next load without a sync).

        A contract-breaking batch (targets not sorted, ids outside [0, N)) is
        only detected on the device: its replay has already run -- on a wrong
        CSR, never out of bounds (the slot kernel stores bad sources as row 0).
        On one rank its optimizer step is skipped on the device (ABI 20: the
        slot's gate word -- parameters, moments and the step count stay as
        they were); with a gradient exchange every rank applies the same
        update, so there the batch has been trained on by the time it is
        reported.  Call this where a training loop ends (the last batch is
        otherwise never reported)."""
        torch.cuda.synchronize(self.x.device)
        self._raise_if_bad()

    def _next_gen(self) -> int:
        self._gen += 1
        if self._gen >= 2**32:  # wrapped: restart the generations from zeroed words
            self.r_next.zero_()
            self._gate.zero_()
            self._gen = 1
        return self._gen

    def _fwd_bwd(self):
        out = self.model(self.x, self.ei)
        # the captured step's logits (static: rewritten by every replay);
        # detached -- holding the warm-up's autograd graph would keep its
        # AccumulateGrad nodes (made on the warm-up stream) alive into the
        # capture: torch's stream-mismatch warning and an event wait per
        # parameter inside the captured backward
        self.out = out.detach()
        # a bf16 model in a slot whose loss reads the seed rows: the bf16
        # logits hold those rows only; every row's logits in fp32 here
        self.out_f32 = getattr(out, "_ngnn_f32", None)
        loss = self.loss_fn(out, self.y, self.B)
        # a persistent d(loss) = 1 instead of backward()'s ones_like fill
        # launch; marked, so the loss backward needs no scale launch either
        if self._one is None or self._one.shape != loss.shape:
            from .losses import unit_grad
            self._one = unit_grad(loss)
        loss.backward(self._one)
        return loss

    def capture(self, x, edge_index, y, restore: bool = True) -> None:
        """Warm up on a side stream (allocates grads, workspaces, optimizer
        state), then capture.  restore=True puts the parameters and optimizer
        state back to their pre-warm-up values afterwards, so graph training
        starts from the same state eager training would."""
        snap = None
        if restore:
            snap = ([p.detach().clone() for p in self.model.parameters()],
                    {k: {n: (t.clone() if torch.is_tensor(t) else t) for n, t in v.items()}
                     for k, v in self.opt.state.items()})
        # bf16 features for a SAGE model: a bf16 slot, read as bf16 by layer 0
        xd = x.table.dtype if isinstance(x, IndexedRows) else x.dtype
        c0 = getattr(getattr(self.model, "convs", [None])[0], "lin_r", None)
        if (xd == torch.bfloat16 and self.x.dtype != torch.bfloat16 and c0 is not None
                and self.x.size(1) % 4 == 0):
            self.x = torch.zeros(self.n_cap, self.x.size(1), dtype=torch.bfloat16,
                                 device=self.x.device)
        self.load(x, edge_index, y)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(self.warmup):
                self.opt.zero_grad(set_to_none=True)
                self._fwd_bwd()
                if self.reducer is not None:
                    self.reducer()
                self.opt.step()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        # the captured Block must be built inside the graph (from the slot's
        # contents at replay time), never served from the eager cache
        block_cache.clear()
        # zero-copy features only where the layer-0 kernel can take them
        # (otherwise every replay copies the rows into the slot)
        from .fused import zero_copy_ok
        table_rows = 0
        if isinstance(x, IndexedRows) and x.table.dtype == torch.float32:
            table_rows = x.table.size(0)
        self.zero_copy = zero_copy_ok(self.model, self.n_cap, self.x.size(1), table_rows)
        if not self.zero_copy and table_rows:  # materialized rows, plain zero-copy if possible
            table_rows = 0
            self.zero_copy = zero_copy_ok(self.model, self.n_cap, self.x.size(1))
        self.x_rows = table_rows if self.zero_copy else 0
        if self.x_rows:
            self.col_x = torch.zeros(self.e_cap, dtype=torch.int32, device=self.x.device)
        self._pack = _prepack_target(self.model)
        # the step's loss taken by a two-layer forward (fused.LossHead): its
        # persistent buffers made here, outside the capture
        self._head = None
        convs = getattr(self.model, "convs", None)
        if (self.loss_fn is seed_cross_entropy and convs is not None and len(convs) == 2
                and self.x.dtype == torch.float32
                and all(_lin_w(c) is not None and _lin_w(c).dtype == torch.float32 for c in convs)):
            from .fused import LossHead
            self._head = LossHead(self.y, self.B, self.n_cap, _lin_w(convs[1]).shape[0], self.r_next)
        hint_edge_index(self.ei, dst_sorted=True, src_sorted=False, n_rows_dev=self.n_valid,
                        csr=CSR(self.rowptr, self.col, self.n_cap), seed_dev=self.seed_state,
                        x_dev=self.x_dev if self.zero_copy else None, r_next=(self.r_next, self.B, self.loss_fn is seed_cross_entropy),
                        n_edge_rows_dev=self.n_edge_rows,
                        xrow=(self.xrow_dev, self.x_rows, self.col_x) if self.x_rows else None,
                        wl_prepacked=self._pack, loss_head=self._head)
        if self._pack is not None:  # the capture's own forward reads it: pack it now
            self.load(x, edge_index, y)
        self.opt.zero_grad(set_to_none=True)
        # the backward's constant row-bound array: created now, not inside the capture
        convs = getattr(self.model, "convs", None)
        if convs is not None:
            from .fused import const_bounds, reserve_sage2_bwd
            const_bounds(self.x.device, len(convs), self.B)
            if len(convs) == 2 and _lin_w(convs[0]) is not None and _lin_w(convs[1]) is not None:
                # (the warm-up ran before the slot's bound hint existed, so it
                # took the per-layer backward: reserve the two-layer one's now)
                reserve_sage2_bwd(self.x.device, self.n_cap, _lin_w(convs[0]).shape[1],
                                  _lin_w(convs[1]).shape[0])
        # data parallel: the bucket pack is the tail of the first graph and the
        # unpack (/ world) the head of the second, so between the replays the
        # host issues only the one all-reduce
        red = self.reducer if (self.reducer is not None and hasattr(self.reducer, "active")
                               and self.reducer.active()) else None
        self._split_reduce = red is not None
        # one rank: the Adam step folds into the two-layer backward's
        # reduction (fused.AdamFoldSpec) -- then no optimizer graph
        from . import fused as _fused
        exchange = red is not None or (self.reducer is not None and not (
            hasattr(self.reducer, "active") and not self.reducer.active()))
        fold = None if exchange else _fused.AdamFoldSpec.make(self.opt, self.model)
        # one rank: a block that broke the slot's contract updates nothing (the
        # gate; with an exchange every rank must apply the same update, so
        # there the error word only reports)
        gate = None if exchange else (self._gate.data_ptr(), self.r_next.data_ptr())
        if fold is not None and gate is not None:
            fold.struct.gate, fold.struct.gate_gen = gate
        self.g_fb = torch.cuda.CUDAGraph()
        _fused._adam_fold = fold
        try:
            with torch.cuda.graph(self.g_fb):
                self.loss = self._fwd_bwd()
                if red is not None:
                    red.pack()
        finally:
            _fused._adam_fold = None
        self.folded = fold is not None and fold.used
        # the replay needs no autograd nodes: holding the captured loss /
        # logits with their graph would keep the capture's AccumulateGrad
        # nodes (made on the capture stream) alive into later eager steps of
        # the same model -- torch's "AccumulateGrad node's stream does not
        # match" warning and an event wait per parameter there
        self.loss = self.loss.detach()
        self.g_opt = None
        if not self.folded:
            from . import optim as _optim
            self.g_opt = torch.cuda.CUDAGraph()
            _optim._slot_gate = gate
            try:
                with torch.cuda.graph(self.g_opt, pool=self.g_fb.pool()):
                    if red is not None:
                        red.unpack()
                    self.opt.step()
            finally:
                _optim._slot_gate = None
        block_cache.clear()
        torch.cuda.synchronize()
        if snap is not None:
            with torch.no_grad():
                for p, v in zip(self.model.parameters(), snap[0]):
                    p.copy_(v)
                for k, st in self.opt.state.items():
                    old = snap[1].get(k)
                    for n, t in st.items():
                        if not torch.is_tensor(t):
                            continue
                        if old is not None and torch.is_tensor(old.get(n)):
                            t.copy_(old[n])
                        else:
                            t.zero_()  # state born in the warm-up: a fresh optimizer's zeros

    def __call__(self, x, edge_index, y, batch_size: int | None = None):
        """Load one batch into the slot and replay the captured step; returns
        the (device) loss tensor of this step.  batch_size: the block's seed
        count when it is short of the captured B (see load)."""
        self.load(x, edge_index, y, zero_copy=self.zero_copy, batch_size=batch_size)
        self.g_fb.replay()
        if self._pack is not None:  # the replayed forward consumed this load's pack
            self._pack[2].armed = False
        if self._split_reduce:
            self.reducer.allreduce()
        elif self.reducer is not None:
            self.reducer()
        if self.g_opt is not None:  # (None: the backward's reduction took the Adam step)
            self.g_opt.replay()
        return self.loss


def _lin_w(conv):
    """The neighbour-term weight of a SAGEConv (lin_l) or GCNConv (lin), else None."""
    lin = getattr(conv, "lin_l", None) or getattr(conv, "lin", None)
    return getattr(lin, "weight", None)


def _prepack_target(model):
    """(W_l, packed buffer) of layer 0 when the model is a fused SAGE stack
    with fp32 weights (a bf16 model's weights are widened copies: no stable
    address), else None."""
    from .fused import pack_weight
    from .models import SAGE
    if not isinstance(model, SAGE) or getattr(model, "use_bn", False):
        return None
    w = model.convs[0].lin_l.weight
    if w.dtype != torch.float32 or not w.is_cuda or w.stride(1) != 1:
        return None
    # the packed W_l at the buffer's head; the layer's workspace size (its
    # tail holds the kernel's prebuilt root image) -- the buffer IS the
    # captured forward's workspace
    from . import _lib
    from . import fused
    Fo, K = w.shape
    lib = _lib.load()
    # layers that never read a pack: the two-layer kernels load
    # their weight slices themselves, the wide path splits W in its own
    # launch -- no pack job in their slot loads
    agg = getattr(model.convs[0], "aggr", "mean")
    c1 = model.convs[-1].lin_l.weight
    if (len(model.convs) == 2 and agg in ("mean", "sum") and c1.dtype == torch.float32
            and fused._use_fwd2 and not fused._exact_f32
            and lib.ngnn_sage2_supported(K, Fo, c1.shape[0], _lib.REDUCE[agg])):
        return None
    if lib.ngnn_sage_wide_preferred(K, Fo, int(fused._exact_f32)):
        return None
    n = max(pack_weight(w.detach()).numel(),
            -(-_lib.load().ngnn_sage_fwd_raw_workspace_bytes(K, Fo, 0) // 4) + 16)
    return (w, torch.zeros(n, dtype=torch.float32, device=w.device), PackState())


class PackState:
    """Validity of the slot's packed W_l: armed by every load() (whose slot
    kernel packed the weight's values of that moment), consumed by the one
    forward that reads it (ngnn.fused._SAGEStack).  A later eager forward over
    the slot -- after an optimizer step, without a new load(), e.g. the
    warm-up's second step -- packs W_l itself instead of reading a stale pack
    (ADVICE r3).  Graph replays are unaffected: each follows its own load."""

    __slots__ = ("armed",)

    def __init__(self):
        self.armed = False


def slot_size(batch_size: int, fanouts, margin_rows: int = 1024):
    """(n_cap, e_cap) for every NeighborLoader block of this shape: the most
    edges the sampler can emit (batch x fanout products) and as many node
    rows plus room for the padding self-loops."""
    e_cap, frontier = 0, int(batch_size)
    for k in fanouts:
        frontier *= int(k)
        e_cap += frontier
    return int(batch_size) + e_cap + margin_rows, e_cap


class GraphedCoTeachingStep(GraphedTrainStep):
    """The co-teaching training loop body (pipeline.py:95-142, ``train_ct``,
    run by ``config_products.yml`` / ``config_amazon.yml``: ``algo_type:
    'coteaching'``) as ONE HIP-graph replay per batch: both models' forwards
    over the slot's block, ``CTLoss`` on their seed rows (per-row cross
    entropies, both argsorts, the exchange selection, the pure ratios --
    ngnn.losses.CTLoss on the device, no host sync), ``loss_1.backward()``,
    ``loss_2.backward()`` and both optimizers' steps.

        step = GraphedCoTeachingStep(model1, opt1, model2, opt2, CTLoss(dev), B, n_cap, e_cap, F,
                                     dev, noise_or_not)
        loss_1, loss_2, pure_ratio_1, pure_ratio_2, _, _, _, _ = step(
            batch.x, batch.edge_index, batch.yhn, batch.n_id, rate_schedule[epoch])

    Returns CTLoss's 8-tuple as device tensors (rewritten by the next replay).  The forget rate
    fixes ``num_remember = int((1 - rate) B)`` (losses.py:29-30), a launch
    argument: one graph per distinct value, captured on first use (the
    reference's schedule has a handful).  The two models draw independent
    dropout masks from the slot seed (``_ngnn_graph_salt``).  A block short
    of the captured batch size (an epoch's last, drop_last off) runs the
    same loop body eagerly, as the reference does (num_remember of its own
    size).  Optimizers: capturable (ngnn.optim.Adam); no Adam fold (two
    models)."""

    def __init__(self, model1, optimizer1, model2, optimizer2, criterion, batch_size: int, n_cap: int,
                 e_cap: int, in_dim: int, device, noise_or_not=None, warmup: int = 3):
        super().__init__(model1, optimizer1, batch_size, n_cap, e_cap, in_dim, device, warmup=warmup)
        if not optimizer2.defaults.get("capturable", False):
            raise ValueError("GraphedCoTeachingStep needs optimizers built with capturable=True")
        self.model2, self.opt2, self.criterion = model2, optimizer2, criterion
        if getattr(model2, "_ngnn_graph_salt", 0) == getattr(model1, "_ngnn_graph_salt", 0):
            model2._ngnn_graph_salt = 0x5DEECE66D  # (independent of model 1's masks)
        dev = torch.device(device)
        self.noise_or_not = None if noise_or_not is None else noise_or_not.to(dev, torch.bool)
        self.ind = torch.zeros(self.B, dtype=torch.int64, device=dev)  # n_id[:B] of the loaded block
        self._graphs: dict = {}  # num_remember -> (graph, CTLoss's 8 outputs)

    def num_remember(self, forget_rate: float, B: int | None = None) -> int:
        return int((1 - forget_rate) * (self.B if B is None else B))

    def _ct_fwd_bwd(self, forget_rate):
        out1 = self.model(self.x, self.ei)
        out2 = self.model2(self.x, self.ei)
        res = self.criterion(out1, out2, self.y, forget_rate, self.ind, self.noise_or_not, batch_size=self.B)
        if self._one is None:
            from .losses import unit_grad
            self._one = unit_grad(res[0])
        res[0].backward(self._one)
        res[1].backward(self._one)
        return tuple(t.detach() if torch.is_tensor(t) else t for t in res)

    def _load_ct(self, x, edge_index, y, n_id, zero_copy: bool) -> None:
        self.load(x, edge_index, y, zero_copy=zero_copy)
        self.ind.copy_(n_id[:self.B])

    def capture(self, x, edge_index, y, n_id=None, forget_rate: float = 0.0, restore: bool = True) -> None:
        """Warm up and capture the graph of num_remember(forget_rate) on this
        block (restore=True: both models and optimizers back to their state
        before the warm-up)."""
        from . import fused as _fused
        from .fused import const_bounds, reserve_sage2_bwd, zero_copy_ok
        models, opts = (self.model, self.model2), (self.opt, self.opt2)
        snap = None
        if restore:
            snap = [([p.detach().clone() for p in m.parameters()],
                     {k: {n: (t.clone() if torch.is_tensor(t) else t) for n, t in v.items()}
                      for k, v in o.state.items()}) for m, o in zip(models, opts)]
        n_id = torch.arange(self.B, device=self.ind.device) if n_id is None else n_id
        self._load_ct(x, edge_index, y, n_id, zero_copy=False)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(self.warmup):
                for o in opts:
                    o.zero_grad(set_to_none=True)
                self._ct_fwd_bwd(forget_rate)
                for o in opts:
                    o.step()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        block_cache.clear()
        self.zero_copy = all(zero_copy_ok(m, self.n_cap, self.x.size(1)) for m in models)
        self.x_rows = 0
        self._pack = None  # (each model packs its own weights inside the graph)
        self._head = None
        hint_edge_index(self.ei, dst_sorted=True, src_sorted=False, n_rows_dev=self.n_valid,
                        csr=CSR(self.rowptr, self.col, self.n_cap), seed_dev=self.seed_state,
                        x_dev=self.x_dev if self.zero_copy else None, r_next=(self.r_next, self.B, True),
                        n_edge_rows_dev=self.n_edge_rows)
        for o in opts:
            o.zero_grad(set_to_none=True)
        for m in models:
            convs = getattr(m, "convs", None)
            if convs is not None:
                const_bounds(self.x.device, len(convs), self.B)
                if len(convs) == 2 and _lin_w(convs[0]) is not None and _lin_w(convs[1]) is not None:
                    reserve_sage2_bwd(self.x.device, self.n_cap, _lin_w(convs[0]).shape[1],
                                      _lin_w(convs[1]).shape[0])
        g = torch.cuda.CUDAGraph()
        pool = next(iter(self._graphs.values()))[0].pool() if self._graphs else None
        _fused._adam_fold = None
        from . import optim as _optim
        _optim._slot_gate = (self._gate.data_ptr(), self.r_next.data_ptr())  # (one rank: the slot's gate)
        try:
            with torch.cuda.graph(g, pool=pool):
                outs = self._ct_fwd_bwd(forget_rate)
                for o in opts:
                    o.step()
        finally:
            _optim._slot_gate = None
        self._graphs[self.num_remember(forget_rate)] = (g, outs)
        block_cache.clear()
        torch.cuda.synchronize()
        if snap is not None:
            with torch.no_grad():
                for (ps, st), m, o in zip(snap, models, opts):
                    for p, v in zip(m.parameters(), ps):
                        p.copy_(v)
                    for k, cur in o.state.items():
                        old = st.get(k)
                        for n, t in cur.items():
                            if not torch.is_tensor(t):
                                continue
                            if old is not None and torch.is_tensor(old.get(n)):
                                t.copy_(old[n])
                            else:
                                t.zero_()

    def __call__(self, x, edge_index, y, n_id, forget_rate: float = 0.0, batch_size: int | None = None):
        """One co-teaching step on a block; returns CTLoss's 8-tuple (loss_1,
        loss_2, pure_ratio_1, pure_ratio_2, ind_1_update, ind_2_update,
        ind_noisy_1, ind_noisy_2; pipeline.py:116) as device tensors.  y: the
        block's noisy labels (batch.yhn, whose first B rows the loss reads);
        n_id: its global ids (CTLoss's ``ind``, for the pure ratios)."""
        bs = self.B if batch_size is None else int(batch_size)
        if bs < self.B:  # a short block: the same loop body, eagerly
            return self._eager(x, edge_index, y, n_id, forget_rate, bs)
        nr = self.num_remember(forget_rate)
        if nr not in self._graphs:
            self.capture(x, edge_index, y, n_id, forget_rate)
        g, outs = self._graphs[nr]
        self._load_ct(x, edge_index, y, n_id, zero_copy=self.zero_copy)
        g.replay()
        return outs

    def _eager(self, x, edge_index, y, n_id, forget_rate, bs):
        x = x.materialize() if isinstance(x, IndexedRows) else x
        out1 = self.model(x, edge_index)
        out2 = self.model2(x, edge_index)
        res = self.criterion(out1, out2, y, forget_rate, n_id, self.noise_or_not, batch_size=bs)
        for o in (self.opt, self.opt2):
            o.zero_grad(set_to_none=False)
        res[0].backward()
        self.opt.step()
        res[1].backward()
        self.opt2.step()
        return tuple(t.detach() if torch.is_tensor(t) else t for t in res)
