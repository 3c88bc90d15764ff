"""Device-resident CSR view of a PyG ``edge_index`` block.

PyG's ``MessagePassing.propagate`` [ext] re-reads ``edge_index`` on every
conv call (``sage.py:34`` runs it once per layer, and autograd runs the
transposed scatter again).  Here an edge_index is validated and grouped by
target ONCE per mini-batch; every layer, the backward pass and the
transposed (by-source) CSR reuse it.

* ``rowptr`` int32 [N+1], ``col`` int32 [E]: edges grouped by target
  (``edge_index[1]``), edge order kept inside a row (stable).
* ``transposed()``: the same grouped by source, for input gradients.

Validation replaces the index errors PyG / ATen raise from ``index_select``:
an out-of-range id raises ``IndexError`` before any kernel touches memory.
That check reads four status words back to the host (one sync per block).
"""
from __future__ import annotations

import collections
import threading
import weakref

import torch

from . import _lib


def _require_device_index(edge_index: torch.Tensor) -> None:
    if not isinstance(edge_index, torch.Tensor):
        raise TypeError("edge_index must be a torch.Tensor (SparseTensor is not supported)")
    if edge_index.dim() != 2 or edge_index.size(0) != 2:
        raise ValueError(f"edge_index must have shape [2, E], got {tuple(edge_index.shape)}")
    if edge_index.dtype != torch.long:
        raise TypeError(f"edge_index must be int64, got {edge_index.dtype}")
    if not edge_index.is_cuda:
        raise RuntimeError("ngnn runs on the GPU only: edge_index is on the CPU "
                           "(move the batch with batch.to(device) as pipeline.py:153 does)")


class CSR:
    __slots__ = ("rowptr", "col", "n_rows", "nnz")

    def __init__(self, rowptr: torch.Tensor, col: torch.Tensor, n_rows: int):
        self.rowptr, self.col, self.n_rows, self.nnz = rowptr, col, n_rows, col.numel()

    def degree(self) -> torch.Tensor:
        return (self.rowptr[1:] - self.rowptr[:-1])


def build_csr(keys: torch.Tensor, vals: torch.Tensor, n_rows: int, keys_sorted: bool) -> CSR:
    lib = _lib.load()
    dev = keys.device
    E = keys.numel()
    rowptr = torch.empty(n_rows + 1, dtype=torch.int32, device=dev)
    col = torch.empty(max(E, 0), dtype=torch.int32, device=dev)
    ws, ws_bytes = None, 0
    if not keys_sorted and E > 0:
        ws_bytes = lib.ngnn_csr_workspace_bytes(E, n_rows)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    rc = lib.ngnn_csr_build(_lib.ptr(keys), _lib.ptr(vals), E, n_rows, int(keys_sorted),
                            _lib.ptr(rowptr), _lib.ptr(col), None, _lib.ptr(ws), ws_bytes,
                            _lib.stream_handle(dev))
    _lib.check(rc, "ngnn_csr_build")
    return CSR(rowptr, col, n_rows)


class Block:
    """Validated, CSR-grouped homogeneous block: ``num_nodes`` sources == targets."""

    def __init__(self, edge_index: torch.Tensor, num_nodes: int, *, n_dst: int | None = None,
                 validate: bool = True, dst_sorted: bool | None = None,
                 src_sorted: bool | None = None, csr: "CSR | None" = None):
        _require_device_index(edge_index)
        edge_index = edge_index.contiguous()
        self.edge_index = edge_index
        self.n_src = int(num_nodes)
        self.n_dst = int(num_nodes if n_dst is None else n_dst)
        self.E = edge_index.size(1)
        self.device = edge_index.device
        if validate or dst_sorted is None or src_sorted is None:
            status = torch.zeros(4, dtype=torch.int32, device=self.device)
            rc = _lib.load().ngnn_edge_probe(_lib.ptr(edge_index), self.E, self.n_src, self.n_dst,
                                             _lib.ptr(status), _lib.stream_handle(self.device))
            _lib.check(rc, "ngnn_edge_probe")
            s = status.tolist()  # host sync: the one validation read-back per block
            if s[0]:
                raise IndexError(f"edge_index[0] holds ids outside [0, {self.n_src})")
            if s[1]:
                raise IndexError(f"edge_index[1] holds ids outside [0, {self.n_dst})")
            dst_sorted, src_sorted = not s[2], not s[3]
        self.dst_sorted, self.src_sorted = bool(dst_sorted), bool(src_sorted)
        # csr: the target-grouped CSR built by a producer (the HIP-graph slot
        # load writes it with the slot's edges), else built here
        self.csr = csr if csr is not None else build_csr(edge_index[1], edge_index[0], self.n_dst,
                                                         self.dst_sorted)
        self._csr_t = None
        self.n_active = None  # leading rows with in-edges, if a producer told us
        # device int32 scalar: rows >= it are padding (a static HIP-graph slot);
        # the forward kernels skip them.  None: every row is real.
        self.n_rows_dev = None
        # device uint64 dropout seed supplied by a producer (graph slot), or None
        self.seed_dev = None
        # device word holding the feature rows' address (zero-copy graph slot:
        # the layer-0 kernels read x there, not from the tensor passed in)
        self.x_dev = None
        # (device int32, R): the input-gradient row bound for output rows < R,
        # kept by a producer (graph slot), or None
        self.r_next = None
        # device int32: rows at or past it have no in-edges (graph slot), or None
        self.n_edge_rows_dev = None
        # fused x[n_id] gather (graph slot): device word holding the address of
        # the batch's n_id (0: x_dev's rows are the block's rows), and the row
        # count of the feature table x_dev then points at
        self.xrow_dev = None
        self.x_rows = 0
        self.col_x = None  # int32 col mapped through n_id (the slot load writes it)
        # (W_l parameter, ngnn_pack_weight(W_l) kept current by a producer) or None
        self.wl_prepacked = None
        # the producer's loss head (ngnn.fused.LossHead: the step's
        # seed_cross_entropy taken by the two-layer forward), or None
        self.loss_head = None

    @property
    def rowptr(self):
        return self.csr.rowptr

    @property
    def col(self):
        return self.csr.col

    def transposed(self) -> CSR:
        """Edges grouped by source (for input gradients); built lazily, cached."""
        if self._csr_t is None:
            ei = self.edge_index
            self._csr_t = build_csr(ei[0], ei[1], self.n_src, self.src_sorted)
        return self._csr_t


class _BlockCache:
    """Tiny LRU keyed by edge_index identity/version, so the layers of one
    forward (and its backward) share one Block.  Holding the tensor keeps its
    storage alive, so a cached data_ptr can never be recycled under us."""

    def __init__(self, capacity: int = 8):
        self.capacity = capacity
        self._d: collections.OrderedDict = collections.OrderedDict()
        self._lock = threading.Lock()

    def get(self, edge_index: torch.Tensor, num_nodes: int) -> Block:
        key = (edge_index.data_ptr(), tuple(edge_index.shape), tuple(edge_index.stride()),
               edge_index._version, int(num_nodes), edge_index.device)
        with self._lock:
            hit = self._d.get(key)
            if hit is not None and hit[0] is edge_index:
                self._d.move_to_end(key)
                return hit[1]
        hint = _hint_for(edge_index)
        if hint is not None:
            blk = Block(edge_index, num_nodes, validate=False, dst_sorted=hint[0],
                        src_sorted=hint[1], csr=hint[4])
            blk.n_active = hint[2]
            blk.n_rows_dev = hint[3]
            blk.seed_dev = hint[5]
            blk.x_dev = hint[6]
            blk.r_next = hint[7]
            blk.n_edge_rows_dev = hint[8]
            if hint[9] is not None:
                blk.xrow_dev, blk.x_rows, blk.col_x = hint[9]
            blk.wl_prepacked = hint[10]
            blk.loss_head = hint[11]
        else:
            blk = Block(edge_index, num_nodes)
        with self._lock:
            self._d[key] = (edge_index, blk)
            while len(self._d) > self.capacity:
                self._d.popitem(last=False)
        return blk

    def clear(self):
        with self._lock:
            self._d.clear()


block_cache = _BlockCache()

# Producer hints: a sampler that builds edge_index itself (ngnn.loader) knows it
# is in range and target-sorted, so the block can skip the validating probe
# (and its host read-back).  Keyed by tensor identity; a weakref guards reuse.
_hints: dict = {}
_hints_lock = threading.Lock()


def hint_edge_index(edge_index: torch.Tensor, *, dst_sorted: bool, src_sorted: bool,
                    n_active: int | None = None, n_rows_dev: torch.Tensor | None = None,
                    csr: CSR | None = None, seed_dev: torch.Tensor | None = None,
                    x_dev: torch.Tensor | None = None, r_next=None,
                    n_edge_rows_dev: torch.Tensor | None = None, xrow=None,
                    wl_prepacked=None, loss_head=None) -> None:
    """n_active: number of leading target rows that can have in-edges (all
    later rows have none) -- only used for roofline accounting.  n_rows_dev:
    device int32 scalar bounding the real rows of a padded slot.  csr: a
    target-grouped CSR of these edges kept current by the producer.
    seed_dev: device uint64 dropout seed the producer advances per batch.
    x_dev: device word the producer fills with the address of the feature
    rows the layer-0 kernels must read (zero-copy slot).  r_next: (device int32,
    R[, trusted]): the producer keeps ngnn_block_prefix_stats' bound for R
    there; trusted: the step's loss reads rows < R only, so a forward may keep
    hidden rows below that bound alone (ngnn.fused.sage2_forward).
    n_edge_rows_dev: device int32 holding n_active for a changing batch.
    xrow: (device word, table rows, col_x): the producer stores the address of
    the batch's n_id in the word when x_dev points at the whole feature table
    (fused x[n_id] gather), 0 otherwise, and keeps col_x = n_id[col] (int32).
    wl_prepacked: (W_l parameter, buffer[, state]) -- the producer keeps the
    buffer = ngnn_pack_weight(W_l) current (the slot load's pack job); state
    (ngnn.graphs.PackState): the pack is current only while state.armed.
    loss_head: ngnn.fused.LossHead -- the producer's loss is
    seed_cross_entropy(out, loss_head.y, loss_head.B) of this block's logits,
    which a two-layer forward may take itself (include/ngnn.h ngnn_xent_head)."""
    ref = weakref.ref(edge_index, lambda _r, k=id(edge_index): _drop_hint(k))
    with _hints_lock:
        _hints[id(edge_index)] = (ref, edge_index._version, dst_sorted, src_sorted, n_active,
                                  n_rows_dev, csr, seed_dev, x_dev, r_next, n_edge_rows_dev, xrow,
                                  wl_prepacked, loss_head)


def _drop_hint(key):
    with _hints_lock:
        _hints.pop(key, None)


def _hint_for(edge_index):
    with _hints_lock:
        h = _hints.get(id(edge_index))
    if h is None or h[0]() is not edge_index or h[1] != edge_index._version:
        return None
    return h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9], h[10], h[11], h[12], h[13]


def get_block(edge_index, num_nodes: int) -> Block:
    if isinstance(edge_index, Block):
        return edge_index
    if getattr(edge_index, "_ngnn_counts", None) is not None:
        # a NeighborLoader(sync_free=True) batch: capacity-sized buffers whose
        # real extent only the device knows (ABI 19)
        raise ValueError("a sync_free NeighborLoader batch feeds GraphedTrainStep only; "
                         "use NeighborLoader(sync_free=False) for eager training")
    return block_cache.get(edge_index, num_nodes)
