"""NeighborLoader contract on the host side (no GPU): the PyG-Data adapter
(pipeline.py:75-83 hands NeighborLoader the dataset's ``data``), the Batch
fields the pipelines read (``x, y, yhn, edge_index, n_id, batch_size``,
pipeline.py:110-118,152-160) and per-rank shard sizes."""
import torch

from ngnn.loader import Batch, Graph, NeighborLoader, graph_from_data


class _Data:
    """Stand-in for torch_geometric.data.Data (attribute access + items())."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    def items(self):
        return self.__dict__.items()


def _data(n=12, e=40, seed=0):
    g = torch.Generator().manual_seed(seed)
    return _Data(x=torch.randn(n, 5, generator=g), y=torch.randint(0, 4, (n, 1), generator=g),
                 yhn=torch.randint(0, 4, (n,), generator=g),
                 train_mask=torch.rand(n, generator=g) < 0.5,
                 edge_index=torch.randint(0, n, (2, e), generator=g), num_nodes=n)


def test_graph_from_data_csc_matches_edge_index():
    d = _data()
    g = graph_from_data(d, device="cpu")
    n = d.num_nodes
    assert g.num_nodes == n and g.num_edges == d.edge_index.size(1)
    # each node's in-neighbours (sources of edges into it) in edge order
    for v in range(n):
        want = d.edge_index[0][d.edge_index[1] == v]
        got = g.col[g.rowptr[v]:g.rowptr[v + 1]].to(torch.int64)
        assert torch.equal(got, want), v
    assert torch.equal(g.y, d.y[:, 0])  # OGB's [N, 1] labels flattened
    assert torch.equal(g.node_attrs["yhn"], d.yhn)
    assert torch.equal(g.train_idx, d.train_mask.nonzero().view(-1))
    assert "x" not in g.node_attrs and "edge_index" not in g.node_attrs


def test_batch_node_attrs_and_to():
    b = Batch(torch.zeros(3, 2), torch.arange(3), torch.zeros(2, 0, dtype=torch.int64),
              torch.tensor([5, 1, 2]), 2, yhn=torch.tensor([0, 1, 1]))
    assert torch.equal(b.yhn, torch.tensor([0, 1, 1]))
    assert b.num_nodes == 3 and b.batch_size == 2
    c = b.to("cpu")
    assert torch.equal(c.yhn, b.yhn) and c.batch_size == 2
    try:
        b.nope
    except AttributeError:
        pass
    else:
        raise AssertionError("unknown attributes must raise AttributeError")


def test_loader_shards_equal_across_ranks():
    n, world, bs = 196_615, 8, 1024  # ogbn-products train seeds over 8 ranks
    g = Graph(torch.zeros(n + 1, dtype=torch.int64), torch.zeros(0, dtype=torch.int32),
              torch.zeros(1, 1), torch.zeros(n, dtype=torch.int64), torch.arange(n), 47)
    lens, sizes, allseeds = set(), set(), []
    for r in range(world):
        ld = NeighborLoader(g, g.train_idx, [15, 10], bs, shuffle=True, seed=7, rank=r,
                            world_size=world)
        s = ld._seeds()
        lens.add(len(ld))
        sizes.add(s.numel())
        allseeds.append(s)
    assert lens == {25} and sizes == {24_577}
    assert torch.equal(torch.cat(allseeds).unique(), torch.arange(n))


def test_indexed_rows_and_zero_copy_envelope():
    """IndexedRows (NeighborLoader(gather_features=False)'s x) behaves as
    table[index] for shape/materialize; the graph slot's zero-copy envelope
    admits a fused x[n_id] gather only within the kernels' offset ranges."""
    import ngnn
    from ngnn.fused import zero_copy_ok
    from ngnn.loader import IndexedRows
    t = torch.randn(50, 8)
    idx = torch.tensor([3, 0, 49, 3])
    r = IndexedRows(t, idx)
    assert r.shape == (4, 8) and r.size(0) == 4 and r.size(1) == 8 and r.dtype == t.dtype
    assert torch.equal(r.materialize(), t[idx])
    assert torch.equal(r.to("cpu").materialize(), t[idx])
    m = ngnn.SAGE(100, 64, 10, 2)
    assert zero_copy_ok(m, 200_000, 100, table_rows=2_449_029)      # ogbn-products table
    assert not zero_copy_ok(m, 200_000, 100, table_rows=6_000_000)  # > 2 GiB (weight gradient)
    # K % 4 (Amazon-Computers' 767): layer 0 runs on the wide path, which
    # reads the rows in place at 4-B alignment -- but never through a fused
    # x[n_id] gather
    assert zero_copy_ok(m, 200_000, 102)
    assert not zero_copy_ok(m, 200_000, 102, table_rows=2_449_029)
    g = ngnn.SimpleGCN(100, 16, 10, 2)  # transform-first layer 0: no zero-copy
    assert not zero_copy_ok(g, 1000, 100)
    assert zero_copy_ok(ngnn.SimpleGCN(100, 256, 10, 2), 1000, 100)


def test_graph_cache_releases_freed_data(monkeypatch):
    """The data -> Graph cache behind NeighborLoader(data, ...) holds its
    data object weakly: the entry (and the device graph it holds) leaves with
    the data object; objects that cannot be weakly referenced are not cached."""
    import gc

    from ngnn import loader
    built = []
    monkeypatch.setattr(loader, "graph_from_data", lambda d: built.append(d) or object())
    d = _data()
    g1 = loader._graph_of(d)
    assert loader._graph_of(d) is g1 and len(built) == 1  # one build per data object
    assert id(d) in loader._graphs_of_data
    key = id(d)
    built.clear()
    del d
    gc.collect()
    assert key not in loader._graphs_of_data
    slots = type("Slots", (), {"__slots__": ("x",)})()  # no __weakref__
    loader._graph_of(slots)
    loader._graph_of(slots)
    assert len(built) == 2 and id(slots) not in loader._graphs_of_data


def test_sync_free_loader_contract_on_the_host():
    """NeighborLoader(sync_free=True) (ABI 19) carries x, y, edge_index and
    n_id only: a graph with further per-node tensors is refused up front; a
    batch marked sync-free (capacity-sized buffers, counts on the device) is
    refused by the models before anything reads it."""
    import pytest

    import ngnn
    d = _data()
    g = graph_from_data(d, device="cpu")
    with pytest.raises(ValueError, match="sync_free"):
        NeighborLoader(g, g.train_idx, [3], 4, sync_free=True)
    g.node_attrs.clear()
    ld = NeighborLoader(g, g.train_idx, [3], 4, sync_free=True)
    assert ld.sync_free and len(ld) == -(-g.train_idx.numel() // 4)
    ei = torch.zeros(2, 8, dtype=torch.int64)
    ei._ngnn_counts = torch.zeros(4, dtype=torch.int32)
    for m in (ngnn.SAGE(5, 8, 4, 2), ngnn.SimpleGCN(5, 8, 4, 2)):
        with pytest.raises(ValueError, match="sync_free"):
            m(torch.zeros(8, 5), ei)
    with pytest.raises(ValueError, match="sync_free"):
        ngnn.SAGEConv(5, 4)(torch.zeros(8, 5), ei)
