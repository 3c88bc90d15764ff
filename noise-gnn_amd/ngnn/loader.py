"""Device-resident graphs and a NeighborLoader-style mini-batch sampler.

The reference builds ``torch_geometric.loader.NeighborLoader`` over an
OGB / PyG dataset (``pipeline.py:75-92``, ``pipeline_s.py:72-89``) whose
sampler (pyg-lib / torch-sparse, C++ [ext]) runs in a worker process and
ships every batch host->device (``pipeline.py:153``).  Here the graph CSR and
the feature table stay resident in HBM and the whole block -- every hop
(uniform, without replacement, Floyd's algorithm), the relabelling to local
ids, the edge list and the x / y gathers -- is built on the GPU by
``ngnn_sample_block``.

Batch layout follows what NeighborLoader hands the model (the contract of
``pipeline.py:152-160``):

* ``n_id``: the seeds first (``[:batch_size]``), then every newly reached
  node of hop 1, then hop 2, ... in order of first appearance;
* ``edge_index`` [2,E] local ids, row 0 = source (sampled neighbour), row 1 =
  target, grouped by target in frontier order => targets non-decreasing;
* ``x = x_all[n_id]``, ``y = y_all[n_id]``, ``batch_size``.

Datasets are not downloadable offline, so :func:`synthetic_graph` makes
seeded graphs with the published sizes of ogbn-products / ogbn-arxiv /
Amazon-Computers / CitationFull-Cora and a power-law
(Chung-Lu) degree profile.
"""
from __future__ import annotations

import dataclasses
import os
import weakref

import torch

from . import _lib
from .block import CSR, hint_edge_index

# name -> (num_nodes, directed entries (symmetric), features, classes, train seeds)
DATASETS = {
    "ogbn-products": (2_449_029, 123_718_280, 100, 47, 196_615),
    "ogbn-arxiv": (169_343, 2_315_598, 128, 40, 90_941),
    "computers": (13_752, 491_722, 767, 10, 300),
    "cora": (19_793, 126_842, 8_710, 70, 1_395),
}


@dataclasses.dataclass
class Graph:
    rowptr: torch.Tensor   # int64 [N+1], in-neighbours of each node (CSC of the symmetric graph)
    col: torch.Tensor      # int32 [nnz]
    x: torch.Tensor        # float32 [N, F]
    y: torch.Tensor        # int64 [N]
    train_idx: torch.Tensor
    num_classes: int
    # further node-level tensors ([N, ...]) every batch carries gathered by
    # n_id, as PyG's NeighborLoader does for each node attribute of `data`
    # (the reference reads batch.yhn, pipeline.py:72,116,157)
    node_attrs: dict = dataclasses.field(default_factory=dict)

    @property
    def num_nodes(self) -> int:
        return self.rowptr.numel() - 1

    @property
    def num_edges(self) -> int:
        return self.col.numel()


class IndexedRows:
    """x[index] without the copy: the rows of ``table`` (a resident feature
    matrix) that a block's ``n_id`` names.  A batch of
    ``NeighborLoader(..., gather_features=False)`` carries one as ``x``; the
    HIP-graph step (ngnn.graphs) hands table and index to the layer-0 kernels,
    which gather the rows themselves (fused x[n_id]); anything else calls
    :meth:`materialize`."""

    def __init__(self, table: torch.Tensor, index: torch.Tensor):
        self.table, self.index = table, index

    @property
    def shape(self):
        return torch.Size((self.index.numel(), self.table.size(1)))

    def size(self, dim=None):
        return self.shape if dim is None else self.shape[dim]

    @property
    def dtype(self):
        return self.table.dtype

    @property
    def device(self):
        return self.table.device

    def to(self, device):
        return IndexedRows(self.table.to(device), self.index.to(device))

    def materialize(self) -> torch.Tensor:
        return self.table.index_select(0, self.index)

    def record_stream(self, stream):
        self.index.record_stream(stream)


class Batch:
    """One NeighborLoader mini-batch: ``x``, ``y``, ``edge_index``, ``n_id``,
    ``batch_size`` and every further node attribute of the graph (``yhn``
    ...) gathered by ``n_id`` -- the fields pipeline.py:110-118,152-160 read."""

    def __init__(self, x, y, edge_index, n_id, batch_size, **node_attrs):
        self.x, self.y, self.edge_index, self.n_id = x, y, edge_index, n_id
        self.batch_size = int(batch_size)
        self.node_attrs = dict(node_attrs)

    def __getattr__(self, name):
        attrs = self.__dict__.get("node_attrs")
        if attrs is not None and name in attrs:
            return attrs[name]
        raise AttributeError(f"Batch has no attribute {name!r}")

    @property
    def num_nodes(self) -> int:
        return self.n_id.numel()

    def to(self, device):
        mv = lambda t: None if t is None else t.to(device)  # noqa: E731
        return Batch(mv(self.x), mv(self.y), mv(self.edge_index), mv(self.n_id), self.batch_size,
                     **{k: mv(v) for k, v in self.node_attrs.items()})


def graph_from_data(data, device=None, train_idx=None, num_classes: int | None = None) -> Graph:
    """Adapter from a PyG-``Data``-like object (the ``data`` the reference
    hands ``NeighborLoader``, pipeline.py:75-83): ``x`` [N, F], ``y`` [N] or
    [N, 1] (OGB), ``edge_index`` [2, E] (row 0 = source, row 1 = target) and
    any further node-level tensors (``yhn`` from flip_label, pipeline.py:72,
    masks ...).  Builds the in-neighbour CSC the device sampler walks (each
    node's sources in edge order, PyG's ``source_to_target`` flow) and moves
    everything to ``device`` once; the feature table stays resident in HBM.
    """
    ei = data.edge_index
    x = data.x
    dev = torch.device(device) if device is not None else (x.device if x.is_cuda else torch.device("cuda"))
    N = int(getattr(data, "num_nodes", None) or x.size(0))
    src, dst = ei[0].to(dev, torch.int64), ei[1].to(dev, torch.int64)
    order = torch.argsort(dst, stable=True)
    counts = torch.bincount(dst, minlength=N)
    rowptr = torch.zeros(N + 1, dtype=torch.int64, device=dev)
    rowptr[1:] = torch.cumsum(counts, 0)
    col = src[order].to(torch.int32)
    y = data.y.to(dev).reshape(N, -1)[:, 0].to(torch.int64).contiguous() \
        if getattr(data, "y", None) is not None else torch.zeros(N, dtype=torch.int64, device=dev)
    if train_idx is None:
        train_idx = getattr(data, "train_idx", None)
        if train_idx is None and getattr(data, "train_mask", None) is not None:
            train_idx = data.train_mask.nonzero().view(-1)
        if train_idx is None:
            train_idx = torch.arange(N)
    skip = {"x", "y", "edge_index", "edge_attr", "train_idx"}
    attrs = {}
    items = data.items() if hasattr(data, "items") else vars(data).items()
    for k, v in items:
        if k in skip or not torch.is_tensor(v) or v.dim() == 0 or v.size(0) != N:
            continue
        attrs[k] = v.to(dev)
    if num_classes is None:
        num_classes = int(getattr(data, "num_classes", 0) or (int(y.max()) + 1 if N else 0))
    return Graph(rowptr, col, x.to(dev).contiguous(), y, train_idx.to(dev), num_classes, attrs)


def _gen(device, seed):
    return torch.Generator(device=device).manual_seed(seed)


def synthetic_graph(name: str = "ogbn-products", device="cuda", seed: int = 0,
                    scale: float = 1.0, num_features: int | None = None) -> Graph:
    """Seeded Chung-Lu graph with the dataset's published N / nnz / F / C.

    ``scale`` < 1 shrinks N and nnz proportionally (tests).  Undirected edges
    are drawn with endpoint probability proportional to a power-law weight
    (w_i ~ (i+1)^-0.5, shuffled), self-loops dropped, then symmetrised, so
    nnz comes out within a fraction of a percent of the target.
    """
    N0, nnz0, F0, C, n_train0 = DATASETS[name]
    N = max(int(N0 * scale), 16)
    nnz = max(int(nnz0 * scale), 32)
    F = num_features or F0
    n_train = max(min(int(n_train0 * scale), N), 1)
    dev = torch.device(device)
    g = _gen(dev, seed)
    w = torch.arange(1, N + 1, device=dev, dtype=torch.float64).pow(-0.5)
    w = w[torch.randperm(N, device=dev, generator=g)]
    cdf = torch.cumsum(w, 0)
    cdf = cdf / cdf[-1]
    m = nnz // 2
    u = torch.searchsorted(cdf, torch.rand(m, device=dev, generator=g, dtype=torch.float64))
    v = torch.searchsorted(cdf, torch.rand(m, device=dev, generator=g, dtype=torch.float64))
    u.clamp_(max=N - 1)
    v.clamp_(max=N - 1)
    keep = u != v
    u, v = u[keep], v[keep]
    src = torch.cat([u, v])
    dst = torch.cat([v, u])
    del u, v, keep
    order = torch.argsort(dst * N + src)
    src, dst = src[order], dst[order]
    del order
    counts = torch.bincount(dst, minlength=N)
    rowptr = torch.zeros(N + 1, dtype=torch.int64, device=dev)
    rowptr[1:] = torch.cumsum(counts, 0)
    col = src.to(torch.int32)
    del src, dst, counts
    gx = _gen(dev, seed + 1)
    x = torch.randn(N, F, device=dev, generator=gx, dtype=torch.float32)
    y = torch.randint(0, C, (N,), device=dev, generator=_gen(dev, seed + 2))
    train_idx = torch.randperm(N, device=dev, generator=_gen(dev, seed + 3))[:n_train]
    return Graph(rowptr, col, x, y, train_idx, C)


def sample_hop(graph: Graph, frontier: torch.Tensor, fanout: int, seed: int):
    """[n_frontier, fanout] global neighbour ids (-1 = none) and counts."""
    nf = frontier.numel()
    out = torch.empty(nf, fanout, dtype=torch.int64, device=frontier.device)
    cnt = torch.empty(nf, dtype=torch.int32, device=frontier.device)
    rc = _lib.load().ngnn_sample_hop(_lib.ptr(graph.rowptr), _lib.ptr(graph.col),
                                     _lib.ptr(frontier), nf, fanout, seed & (2**64 - 1),
                                     _lib.ptr(out), _lib.ptr(cnt),
                                     _lib.stream_handle(frontier.device))
    _lib.check(rc, "ngnn_sample_hop")
    return out, cnt


class _SamplerState:
    """One set of ngnn_sample_block's device state: the node map (int32
    [2 N], all -1 between blocks), one workspace per (batch, fanouts) and two
    count slots (the loader reads batch b's counts while batch b + 1 is being
    sampled into the other slot).  A set serves one block in flight at a
    time: a NeighborLoader iterator leases one for its whole pass (it keeps
    a block sampled ahead), so two live iterators never share a node map."""

    def __init__(self, n: int, device):
        self.node_map = torch.full((2 * n,), -1, dtype=torch.int32, device=device)
        self.ws: dict = {}
        self.counts = torch.empty(2, 4, dtype=torch.int32, device=device)
        self.counts_host = torch.empty(2, 4, dtype=torch.int32).pin_memory()
        self.released = None  # event after the last launch of the previous lease

    def outputs(self, batch: int, fan, n_hops: int, x: torch.Tensor | None):
        """Capacity-sized output buffers of a sync-free block (ABI 19): n_id,
        edge_index [2, e_cap], y, x rows (when gathered) and the device
        counts -- written by the finish launch with the block's counts read on
        the device, reused by every block this state samples."""
        e_cap, nf = 0, int(batch)
        for h in range(n_hops):
            nf *= int(fan[h])
            e_cap += nf
        n_cap = int(batch) + e_cap
        key = ("out", batch, tuple(fan[:n_hops]), None if x is None else (x.size(1), x.dtype))
        buf = self.ws.get(key)
        if buf is None:
            dev = self.node_map.device
            # (n_id zero-filled once: entries past a block's count always hold
            # valid node ids -- 0 or an earlier block's -- so nothing that
            # indexes with the whole buffer can leave the table)
            buf = (torch.zeros(n_cap, dtype=torch.int64, device=dev),
                   torch.empty(2, max(e_cap, 1), dtype=torch.int64, device=dev)[:, :e_cap],
                   torch.empty(n_cap, dtype=torch.int64, device=dev),
                   None if x is None else torch.empty(n_cap, x.size(1), dtype=x.dtype, device=dev),
                   torch.zeros(4, dtype=torch.int32, device=dev), n_cap, e_cap)
            self.ws[key] = buf
        return buf

    def workspace(self, lib, batch: int, fan, n_hops: int) -> torch.Tensor:
        key = (batch, tuple(fan[:n_hops]))
        buf = self.ws.get(key)
        if buf is None:
            n = lib.ngnn_sample_block_workspace_bytes(batch, fan, n_hops)
            if n == 0:
                raise ValueError(f"unsupported sampling shape: batch {batch}, "
                                 f"fanouts {list(fan[:n_hops])} (each 0..64, at most 8 hops)")
            buf = torch.empty(n, dtype=torch.uint8, device=self.node_map.device)
            self.ws[key] = buf
        return buf


class _SamplerCache:
    """Per-graph pool of sampler state sets, leased on the current stream
    (which first waits for the set's previous lease to finish on its own)."""

    def __init__(self, n: int, device):
        self.n, self.device = n, device
        self.free: list = []

    def acquire(self) -> _SamplerState:
        st = self.free.pop() if self.free else _SamplerState(self.n, self.device)
        if st.released is not None:
            torch.cuda.current_stream(self.device).wait_event(st.released)
        return st

    def release(self, st: _SamplerState) -> None:
        st.released = torch.cuda.Event()
        st.released.record(torch.cuda.current_stream(self.device))
        self.free.append(st)


_sampler_caches: dict = {}


def _sampler_cache(graph: Graph) -> _SamplerCache:
    key = (graph.col.data_ptr(), graph.num_nodes, graph.col.device)
    c = _sampler_caches.get(key)
    if c is None:
        c = _SamplerCache(graph.num_nodes, graph.col.device)
        _sampler_caches[key] = c
    return c


class _Pending:
    """A block whose sampling kernels are enqueued (ngnn_sample_block) and
    whose counts are on their way to pinned host memory (``event``)."""

    __slots__ = ("graph", "state", "ws", "fan", "H", "B", "slot", "event", "gather_features", "seeds")


def _sample_start(graph: Graph, seeds: torch.Tensor, fanouts, seed: int, gather_features: bool,
                  state: _SamplerState, slot: int = 0) -> _Pending:
    """Enqueue the sampling of one block on the current stream: every hop,
    the relabelling and the edge list (ngnn_sample_block), then an async
    copy of its (node, edge, active-row) counts into count slot `slot`."""
    import ctypes
    lib = _lib.load()
    dev = seeds.device
    if not seeds.is_cuda:
        raise RuntimeError("ngnn.loader.sample_block: GPU only (no CPU fallback)")
    if graph.y.dtype != torch.int64 or not graph.y.is_contiguous():
        raise TypeError("graph.y must be a contiguous int64 vector")
    if gather_features and (graph.x.dtype not in (torch.float32, torch.bfloat16)
                            or graph.x.stride(1) != 1
                            or (graph.x.dtype == torch.bfloat16 and graph.x.size(1) % 2)):
        raise TypeError("graph.x must be a row-major float32 matrix (or bf16 with an even width)")
    s64 = seeds.to(torch.int64).contiguous()
    p = _Pending()
    p.graph, p.B, p.H, p.slot, p.gather_features, p.seeds = graph, s64.numel(), len(fanouts), slot, gather_features, s64
    p.fan = (ctypes.c_int32 * max(len(fanouts), 1))(*[int(k) for k in fanouts])
    p.state = state
    p.ws = state.workspace(lib, p.B, p.fan, p.H)
    _lib.check(lib.ngnn_sample_block(
        _lib.ptr(graph.rowptr), _lib.ptr(graph.col), graph.num_nodes, _lib.ptr(s64), p.B, p.fan, p.H,
        int(seed) & (2**64 - 1), _lib.ptr(state.node_map), _lib.ptr(p.ws), p.ws.numel(),
        _lib.ptr(state.counts[slot]), _lib.stream_handle(dev)), "ngnn_sample_block")
    state.counts_host[slot].copy_(state.counts[slot], non_blocking=True)
    p.event = torch.cuda.Event()
    p.event.record(torch.cuda.current_stream(dev))
    return p


def sample_block(graph: Graph, seeds: torch.Tensor, fanouts, seed: int,
                 gather_features: bool = True) -> Batch:
    """One NeighborLoader mini-batch (pipeline.py:152-160 contract) sampled,
    relabelled and gathered on the device by ngnn_sample_block (+ _finish):
    about a dozen launches and ONE device->host read (the block's node and
    edge counts, needed to size the outputs).  Seeds must be distinct.
    (NeighborLoader reads those counts one batch late instead: no wait.)"""
    cache = _sampler_cache(graph)
    st = cache.acquire()
    # (a state set whose block failed half way may hold a node map that was
    # never reset: it is dropped, not returned to the pool)
    blk = _sample_finish(_sample_start(graph, seeds, fanouts, seed, gather_features, st))
    cache.release(st)
    return blk


def _sample_finish(p: _Pending) -> Batch:
    """Wait for the block's counts (its sampling kernels only), then enqueue
    the outputs on the current stream: n_id, edge_index, y, x = x_all[n_id]
    (the finish launch, which also resets the sampler's node map)."""
    lib = _lib.load()
    graph, cache, ws, fan, H, B = p.graph, p.state, p.ws, p.fan, p.H, p.B
    dev = p.seeds.device
    st = _lib.stream_handle(dev)
    gather_features = p.gather_features
    p.event.synchronize()
    n, e, n_active = (int(v) for v in cache.counts_host[p.slot, :3])
    n_id = torch.empty(n, dtype=torch.int64, device=dev)
    edge_index = torch.empty(2, e, dtype=torch.int64, device=dev)
    y = torch.empty(n, dtype=torch.int64, device=dev)
    x = xw = None
    xa = graph.x
    if gather_features:
        x = torch.empty(n, graph.x.size(1), dtype=graph.x.dtype, device=dev)
        # the row gather copies 32-bit words: bf16 rows are viewed as float32 pairs
        xa = graph.x.view(torch.float32) if graph.x.dtype == torch.bfloat16 else graph.x
        xw = x.view(torch.float32) if x.dtype == torch.bfloat16 else x
    # the block's CSR comes out of the relabelling (no CSR build in the model's forward)
    rowptr = torch.empty(n + 1, dtype=torch.int32, device=dev)
    col = torch.empty(max(e, 0), dtype=torch.int32, device=dev)
    _lib.check(lib.ngnn_sample_block_finish(
        fan, H, B, n, e, _lib.ptr(cache.node_map), graph.num_nodes, _lib.ptr(ws), ws.numel(),
        _lib.ptr(n_id), _lib.ptr(edge_index), _lib.ptr(graph.y), _lib.ptr(y), _lib.ptr(xa),
        xa.stride(0), xa.size(1), _lib.ptr(xw), xw.stride(0) if xw is not None else 0, n_active,
        _lib.ptr(rowptr), _lib.ptr(col), None, st), "ngnn_sample_block_finish")
    # built here: ids are in range and targets non-decreasing -> no probe needed
    hint_edge_index(edge_index, dst_sorted=True, src_sorted=False, n_active=n_active,
                    csr=CSR(rowptr, col, n))
    # further node attributes (batch.yhn ...): one device gather each, on this stream
    extra = {k: v.index_select(0, n_id) for k, v in graph.node_attrs.items()}
    return Batch(x, y, edge_index, n_id, B, **extra)


def _sample_sync_free(graph: Graph, seeds: torch.Tensor, fanouts, seed: int, gather_features: bool,
                      state: _SamplerState) -> Batch:
    """One block sampled into the state's capacity-sized buffers with no
    host read-back (ABI 19): ngnn_sample_block writes the counts on the
    device, the finish launch reads them there.  The batch's tensors are
    those buffers (rows / edges past the block's counts are stale) and its
    edge_index carries the device counts (``_ngnn_counts``) for
    GraphedTrainStep.load, the one consumer of such a batch."""
    import ctypes
    lib = _lib.load()
    dev = seeds.device
    s64 = seeds.to(torch.int64).contiguous()
    B, H = s64.numel(), len(fanouts)
    fan = (ctypes.c_int32 * max(H, 1))(*[int(k) for k in fanouts])
    ws = state.workspace(lib, B, fan, H)
    xa = graph.x if gather_features else None
    n_id, ei, y, x, cnt, n_cap, e_cap = state.outputs(B, fan, H, xa)
    st = _lib.stream_handle(dev)
    _lib.check(lib.ngnn_sample_block(
        _lib.ptr(graph.rowptr), _lib.ptr(graph.col), graph.num_nodes, _lib.ptr(s64), B, fan, H,
        int(seed) & (2**64 - 1), _lib.ptr(state.node_map), _lib.ptr(ws), ws.numel(), _lib.ptr(cnt), st),
        "ngnn_sample_block")
    xw = xaw = None
    if gather_features:
        xaw = xa.view(torch.float32) if xa.dtype == torch.bfloat16 else xa
        xw = x.view(torch.float32) if x.dtype == torch.bfloat16 else x
    _lib.check(lib.ngnn_sample_block_finish(
        fan, H, B, n_cap, e_cap, _lib.ptr(state.node_map), graph.num_nodes, _lib.ptr(ws), ws.numel(),
        _lib.ptr(n_id), _lib.ptr(ei), _lib.ptr(graph.y), _lib.ptr(y), _lib.ptr(xaw),
        xaw.stride(0) if xaw is not None else 0, xaw.size(1) if xaw is not None else 0, _lib.ptr(xw),
        xw.stride(0) if xw is not None else 0, 0, None, None, _lib.ptr(cnt), st), "ngnn_sample_block_finish")
    ei._ngnn_counts = cnt
    return Batch(x if gather_features else IndexedRows(graph.x, n_id), y, ei, n_id, B)


# id(data) -> (weakref to data, Graph); an entry leaves with its data object
# (the weakref's callback), so the device copies of a freed data object's
# features and CSR are released with it
_graphs_of_data: dict = {}


def _forget_graph(key, ref) -> None:
    hit = _graphs_of_data.get(key)
    if hit is not None and hit[0] is ref:  # (not an entry of a later object with the same id)
        del _graphs_of_data[key]


def _graph_of(data) -> Graph:
    """graph_from_data once per data object (the reference builds a train and
    a subgraph loader over the same data, pipeline.py:75-92).  Objects that
    cannot be weakly referenced are not cached (a strong reference would keep
    them, and their device graph, alive for the life of the process)."""
    key = id(data)
    hit = _graphs_of_data.get(key)
    if hit is not None and hit[0]() is data:
        return hit[1]
    g = graph_from_data(data)
    try:
        ref = weakref.ref(data, lambda r, k=key: _forget_graph(k, r))
    except TypeError:
        return g
    _graphs_of_data[key] = (ref, g)
    return g


class NeighborLoader:
    """Iterable of :class:`Batch` over ``input_nodes`` (default: all nodes).

    Mirrors the ``NeighborLoader(data, input_nodes, num_neighbors, batch_size,
    shuffle)`` arguments of pipeline.py:75-92; ``num_workers`` /
    ``persistent_workers`` have no meaning here (sampling runs on the GPU).
    ``rank`` / ``world_size`` shard the (shuffled) seeds for seed-node data
    parallelism: every rank draws the same permutation and takes its slice.
    """

    def __init__(self, graph, input_nodes=None, num_neighbors=(15, 10), batch_size=1024,
                 shuffle=False, seed: int = 0, rank: int = 0, world_size: int = 1,
                 drop_last: bool = False, gather_features: bool = True, sync_free: bool = False,
                 **_ignored):
        if not isinstance(graph, Graph):  # the reference's `data` (pipeline.py:75-92)
            graph = _graph_of(graph)
        self.graph = graph
        dev = graph.rowptr.device
        if input_nodes is None:
            input_nodes = torch.arange(graph.num_nodes, device=dev)
        self.input_nodes = input_nodes.to(dev)
        self.num_neighbors = list(num_neighbors)
        self.batch_size = int(batch_size)
        self.shuffle, self.seed = shuffle, seed
        self.rank, self.world_size = rank, world_size
        self.drop_last = drop_last
        # False: batches carry x = IndexedRows(graph.x, n_id) (no row copy)
        self.gather_features = gather_features
        # True (ABI 19): no host read-back per batch -- blocks land in
        # capacity-sized buffers with their counts on the device, for
        # GraphedTrainStep only (see __iter__)
        self.sync_free = sync_free
        if sync_free and graph.node_attrs:
            raise ValueError("sync_free batches carry x, y, edge_index and n_id only")
        self.epoch = 0

    def _seeds(self):
        # every rank gets the same number of seeds (the permutation is padded
        # cyclically when world_size does not divide it), so every rank runs
        # the same number of steps and gradient all-reduces per epoch
        from .distributed import shard_seeds
        return shard_seeds(self.input_nodes, self.rank, self.world_size, self.epoch, self.seed,
                           shuffle=self.shuffle)

    def __len__(self):
        from .distributed import shard_len
        n = shard_len(self.input_nodes.numel(), self.world_size)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __iter__(self):
        """Batches are sampled on a side stream, one batch AHEAD: when the
        consumer asks for batch b, batch b's sampling kernels were enqueued
        during the previous request, so the host waits only for those (never
        for a training step in flight) to read b's sizes, enqueues b's output
        launch and batch b + 1's sampling, and hands b over -- the main stream
        waits for b's outputs alone.  Sampling overlaps training the way the
        reference's worker process overlaps it (pipeline.py:81-82), with no
        per-batch drain of the consumer's stream.  The per-batch seeds follow
        the batch index, so the batches are those of one-at-a-time sampling."""
        seeds = self._seeds()
        ep = self.epoch
        self.epoch += 1
        dev = seeds.device
        main = torch.cuda.current_stream(dev)
        # (NGNN_SIDE_PRIORITY: the sampling stream's priority, torch's scale --
        # negative is higher; A/B of how its kernels share the device with
        # the step's)
        side = torch.cuda.Stream(dev, priority=int(os.environ.get("NGNN_SIDE_PRIORITY", "0")))
        side.wait_stream(main)  # seeds (randperm) were made on the main stream
        n = len(self)
        cache = _sampler_cache(self.graph)
        if self.sync_free:
            yield from self._iter_sync_free(seeds, ep, n, main, side, cache)
            return
        with torch.cuda.stream(side):
            state = cache.acquire()  # this pass's node map / workspace / count slots

        def start(b):
            s = seeds[b * self.batch_size:(b + 1) * self.batch_size]
            with torch.cuda.stream(side):
                return _sample_start(self.graph, s, self.num_neighbors,
                                     seed=(self.seed * 7919 + ep) * 100_003 + b * self.world_size + self.rank,
                                     gather_features=self.gather_features, state=state, slot=b & 1)

        pending = None
        try:
            pending = start(0) if n else None
            for b in range(n):
                with torch.cuda.stream(side):
                    blk = _sample_finish(pending)  # (waits for batch b's counts only)
                    pending = None
                    if not self.gather_features:
                        blk.x = IndexedRows(self.graph.x, blk.n_id)
                    ready = torch.cuda.Event()
                    ready.record(side)
                # the next block's sampling behind this one's outputs (the node
                # map is reset by the finish launch, stream-ordered before it)
                pending = start(b + 1) if b + 1 < n else None
                main.wait_event(ready)
                for t in (blk.x, blk.y, blk.edge_index, blk.n_id, *blk.node_attrs.values()):
                    if t is not None:
                        t.record_stream(main)  # consumed on the main stream
                yield blk
        finally:
            # a pass left early (break, close, garbage collection) still holds
            # a block sampled ahead: finish it, which resets the node map,
            # before the state set goes back to the pool (a set whose finish
            # raised is dropped instead: its node map may not be clean)
            with torch.cuda.stream(side):
                if pending is not None:
                    _sample_finish(pending)
                cache.release(state)

    def _iter_sync_free(self, seeds, ep, n, main, side, cache):
        """sync_free passes (ABI 19): no host wait at all.  Two leased state
        sets alternate; block b is sampled on the side stream into set b & 1
        once the consumer's work on block b - 2 (which read that set's
        buffers) is done -- an event, not a host wait -- and the main stream
        waits for block b's outputs.  The host only enqueues, so it runs
        ahead of the device and sampling overlaps the previous step.  The
        batches' tensors are the sets' capacity-sized buffers with the
        counts on the device (edge_index._ngnn_counts): GraphedTrainStep
        consumes them; an eager model refuses them (ngnn.block.get_block).
        A batch's contents are valid until two batches later."""
        states, done = [], [None, None]
        try:
            with torch.cuda.stream(side):
                states = [cache.acquire(), cache.acquire()]
            for b in range(n):
                s = seeds[b * self.batch_size:(b + 1) * self.batch_size]
                with torch.cuda.stream(side):
                    if done[b & 1] is not None:
                        side.wait_event(done[b & 1])
                    blk = _sample_sync_free(self.graph, s, self.num_neighbors,
                                            (self.seed * 7919 + ep) * 100_003 + b * self.world_size + self.rank,
                                            self.gather_features, states[b & 1])
                    ready = torch.cuda.Event()
                    ready.record(side)
                main.wait_event(ready)
                yield blk
                ev = torch.cuda.Event()
                ev.record(main)  # after the consumer's launches on block b
                done[b & 1] = ev
        finally:
            with torch.cuda.stream(side):
                for ev in done:
                    if ev is not None:
                        side.wait_event(ev)
                for st in states:
                    cache.release(st)
