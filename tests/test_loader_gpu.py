"""GPU neighbour sampler + NeighborLoader batch contract (pipeline.py:152-160):
seeds first, target-sorted local edges, each sampled edge a real graph edge,
min(deg, fanout) distinct neighbours per frontier node, uniform selection."""
import numpy as np
import pytest
import torch

from ngnn.loader import NeighborLoader, sample_block, sample_hop, synthetic_graph

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def graph():
    return synthetic_graph("ogbn-arxiv", DEV, seed=0, scale=0.05)


def test_synthetic_graph_shape(graph):
    N = graph.num_nodes
    assert graph.rowptr[0] == 0 and graph.rowptr[-1] == graph.num_edges
    col = graph.col.long()
    assert int(col.min()) >= 0 and int(col.max()) < N
    # symmetric: multiset of (u,v) == multiset of (v,u)
    dst = torch.repeat_interleave(torch.arange(N, device=DEV), graph.rowptr.diff())
    a = torch.sort(col * N + dst).values
    b = torch.sort(dst * N + col).values
    assert torch.equal(a, b)
    assert abs(graph.num_edges / (2_315_598 * 0.05) - 1) < 0.01


def test_sample_hop_contract(graph):
    frontier = torch.arange(0, graph.num_nodes, 7, device=DEV)
    k = 10
    nbr, cnt = sample_hop(graph, frontier, k, seed=42)
    rp = graph.rowptr.cpu().numpy()
    col = graph.col.cpu().numpy()
    nbr, cnt, fr = nbr.cpu().numpy(), cnt.cpu().numpy(), frontier.cpu().numpy()
    for i in range(0, len(fr), 13):
        v = fr[i]
        adj = col[rp[v]:rp[v + 1]]
        d = len(adj)
        assert cnt[i] == min(d, k)
        got = nbr[i, :cnt[i]]
        assert (nbr[i, cnt[i]:] == -1).all()
        # each draw is a distinct CSR position; values are real neighbours
        assert np.isin(got, adj).all()
        if d <= k:
            assert np.array_equal(got, adj)
    # determinism
    nbr2, _ = sample_hop(graph, frontier, k, seed=42)
    assert np.array_equal(nbr2.cpu().numpy(), nbr)


def test_sample_hop_uniform():
    # star: node 0 has 40 in-neighbours 1..40; sample 5 many times
    N = 41
    rowptr = torch.zeros(N + 1, dtype=torch.int64)
    rowptr[1:] = 40
    col = torch.arange(1, 41, dtype=torch.int32)
    from ngnn.loader import Graph
    g = Graph(rowptr.to(DEV), col.to(DEV), torch.zeros(N, 1, device=DEV),
              torch.zeros(N, dtype=torch.long, device=DEV), torch.arange(1, device=DEV), 1)
    frontier = torch.zeros(20000, dtype=torch.int64, device=DEV)
    nbr, cnt = sample_hop(g, frontier, 5, seed=7)
    assert (cnt == 5).all()
    nb = nbr.cpu().numpy()
    assert all(len(set(r)) == 5 for r in nb[:500])
    hist = np.bincount(nb.ravel(), minlength=41)[1:]
    exp = 20000 * 5 / 40
    chi2 = ((hist - exp) ** 2 / exp).sum()
    assert chi2 < 100, chi2  # 39 dof; p ~ 1e-7 at 100


def test_block_layout(graph):
    seeds = graph.train_idx[:300]
    b = sample_block(graph, seeds, [15, 10], seed=5)
    assert b.batch_size == 300
    assert torch.equal(b.n_id[:300], seeds)
    assert b.n_id.unique().numel() == b.n_id.numel()
    src, dst = b.edge_index
    assert int(src.max()) < b.num_nodes and int(dst.max()) < b.num_nodes
    assert bool((dst[1:] >= dst[:-1]).all()), "targets must be non-decreasing"
    # every local edge maps to a real graph edge (u -> v means u in N_in(v))
    gs, gd = b.n_id[src].cpu().numpy(), b.n_id[dst].cpu().numpy()
    rp, col = graph.rowptr.cpu().numpy(), graph.col.cpu().numpy()
    for u, v in list(zip(gs, gd))[::97]:
        assert u in col[rp[v]:rp[v + 1]]
    # hop-1 targets are seeds; fanout respected
    deg = torch.bincount(dst, minlength=b.num_nodes)
    assert int(deg[:300].max()) <= 15 and int(deg[300:].max()) <= 10
    torch.testing.assert_close(b.x, graph.x[b.n_id])


def test_loader_epoch_and_sharding(graph):
    ld = NeighborLoader(graph, graph.train_idx, [5, 5], batch_size=512, shuffle=True, seed=1)
    seen = torch.cat([b.n_id[:b.batch_size] for b in ld])
    assert torch.equal(seen.sort().values, graph.train_idx.sort().values)
    # two ranks partition the same permutation
    parts = []
    for r in range(2):
        l2 = NeighborLoader(graph, graph.train_idx, [5], batch_size=512, shuffle=True, seed=1,
                            rank=r, world_size=2)
        parts.append(torch.cat([b.n_id[:b.batch_size] for b in l2]))
    both = torch.cat(parts)
    # equal shards: the odd count is padded cyclically (every rank the same
    # number of batches, hence of gradient all-reduces), covering every seed
    n = graph.train_idx.numel()
    assert parts[0].numel() == parts[1].numel() == -(-n // 2)
    assert torch.equal(both.unique(), graph.train_idx.unique())


# ---- native whole-block sampler (ngnn_sample_block) vs the torch restatement

from sampler_ref import sample_block_ref  # noqa: E402


def _assert_same_block(b, ref):
    assert torch.equal(b.n_id, ref.n_id)
    assert torch.equal(b.edge_index, ref.edge_index)
    assert torch.equal(b.y, ref.y)
    assert torch.equal(b.x, ref.x)
    assert b.batch_size == ref.batch_size


@pytest.mark.parametrize("fanouts,bs", [([15, 10], 300), ([5], 64), ([20, 15, 10], 128),
                                        ([3, 0, 2], 50), ([64], 17), ([], 10),
                                        ([2, 2, 2, 2, 2, 2, 2, 2], 8), ([33, 9], 40)])
def test_sample_block_matches_reference(graph, fanouts, bs):
    from ngnn.loader import _sampler_cache
    seeds = graph.train_idx[:bs]
    for s in (1, 99):
        b = sample_block(graph, seeds, fanouts, seed=s)
        ref, n_active = sample_block_ref(graph, seeds, fanouts, s)
        _assert_same_block(b, ref)
        from ngnn.block import _hint_for, build_csr
        assert _hint_for(b.edge_index)[2] == n_active
        # ABI 18: the sampler's own CSR of the block == the one a build makes
        csr = _hint_for(b.edge_index)[4]
        ref_csr = build_csr(b.edge_index[1], b.edge_index[0], b.num_nodes, True)
        assert torch.equal(csr.rowptr, ref_csr.rowptr) and torch.equal(csr.col, ref_csr.col)
    # the node map is restored after every block
    assert all(bool((st.node_map == -1).all()) for st in _sampler_cache(graph).free)


def test_loader_pass_suspended_or_abandoned(graph):
    """The loader samples one batch ahead (no host wait on the consumer's
    stream).  A pass left suspended with a block in flight -- bench.py
    pre-samples a few batches, then runs a whole epoch -- or abandoned must
    not disturb another pass over the same graph: every pass leases its own
    node map.  Every batch equals the synchronous sample_block of the same
    seeds and seed; after the passes end, every node map is clean."""
    from ngnn.distributed import shard_seeds
    from ngnn.loader import _sampler_cache
    ld = NeighborLoader(graph, graph.train_idx, [15, 10], batch_size=256, shuffle=True, seed=3)

    def expect(ep, b):
        s = shard_seeds(ld.input_nodes, 0, 1, ep, ld.seed, shuffle=True)[b * 256:(b + 1) * 256]
        return sample_block(graph, s, [15, 10], seed=(ld.seed * 7919 + ep) * 100_003 + b)

    it = iter(ld)  # epoch 0
    got0 = [next(it) for _ in range(2)]  # suspended: batch 2 in flight
    got1 = list(ld)  # epoch 1, a whole pass meanwhile
    got0.append(next(it))
    it.close()  # abandoned with batch 3 in flight
    torch.cuda.synchronize()
    for b, blk in enumerate(got0):
        _assert_same_block(blk, expect(0, b))
    assert len(got1) == len(ld)
    for b in (0, 1, len(got1) - 1):
        _assert_same_block(got1[b], expect(1, b))
    assert all(bool((st.node_map == -1).all()) for st in _sampler_cache(graph).free)


def test_sample_block_multigraph_and_isolated():
    """duplicate edges (the same neighbour at two CSR positions), a seed with
    no in-edges, degree < fanout, and a self loop."""
    from ngnn.loader import Graph
    # node: in-neighbours
    adj = {0: [1, 1, 2, 3, 4, 5, 6, 1], 1: [], 2: [2, 0], 3: [0, 1, 2, 4, 5, 6, 7, 8, 9],
           4: [9], 5: [0, 0, 0], 6: [], 7: [3], 8: [8, 8], 9: [1, 2, 3, 4]}
    N = 10
    rowptr = [0]
    col = []
    for v in range(N):
        col += adj[v]
        rowptr.append(len(col))
    g = Graph(torch.tensor(rowptr, device=DEV), torch.tensor(col, dtype=torch.int32, device=DEV),
              torch.randn(N, 12, device=DEV), torch.arange(N, device=DEV) % 3,
              torch.arange(N, device=DEV), 3)
    for seeds in ([0, 1, 3], [6, 1], [9, 8, 7, 5]):
        s = torch.tensor(seeds, device=DEV)
        for fan in ([4, 3], [2, 2, 2], [10]):
            for sd in range(4):
                b = sample_block(g, s, fan, seed=sd)
                ref, _ = sample_block_ref(g, s, fan, sd)
                _assert_same_block(b, ref)


def test_sample_block_full_products_size():
    """a products-shaped [15,10] bs=1024 block at full graph size: the native
    block equals the restatement and respects the capacity bounds."""
    g = synthetic_graph("ogbn-products", DEV, seed=0, scale=0.25)
    seeds = g.train_idx[:1024]
    b = sample_block(g, seeds, [15, 10], seed=12345)
    ref, _ = sample_block_ref(g, seeds, [15, 10], 12345)
    _assert_same_block(b, ref)
    assert b.num_nodes <= 1024 * (1 + 15 + 150) and b.edge_index.size(1) <= 1024 * 165


def test_loader_from_data_object_carries_yhn():
    """NeighborLoader(data, ...) as pipeline.py:75-83 builds it: a PyG-Data-
    like object with x, y [N, 1], yhn and edge_index; every batch carries
    yhn = yhn_all[n_id] (pipeline.py:116,157) and y = y_all[n_id]."""

    class _Data:
        def __init__(self, **kw):
            self.__dict__.update(kw)

        def items(self):
            return self.__dict__.items()

    g = synthetic_graph("ogbn-arxiv", DEV, seed=4, scale=0.02)
    N = g.num_nodes
    dst = torch.repeat_interleave(torch.arange(N, device=DEV), g.rowptr.diff())
    ei = torch.stack([g.col.long(), dst]).cpu()
    yhn = torch.randint(0, 40, (N,))
    data = _Data(x=g.x.cpu(), y=g.y.cpu().view(-1, 1), yhn=yhn, edge_index=ei, num_nodes=N)
    loader = NeighborLoader(data, input_nodes=g.train_idx.cpu(), num_neighbors=[10, 5],
                            batch_size=128, shuffle=True)
    n = 0
    for b in loader:
        assert torch.equal(b.yhn.cpu(), yhn[b.n_id.cpu()])
        assert torch.equal(b.y.cpu(), data.y[b.n_id.cpu(), 0])
        assert torch.equal(b.x.cpu(), data.x[b.n_id.cpu()])
        n += 1
        if n == 3:
            break
    assert n == 3


def test_sync_free_batches_equal_the_synchronous_ones(graph):
    """NeighborLoader(sync_free=True) (ABI 19): no host read-back per batch --
    the blocks land in capacity-sized buffers with their counts on the
    device.  Read back here, every batch's first n rows / E edges equal the
    same pass of the synchronous loader bit for bit, for both feature modes;
    an eager model refuses such a batch."""
    import ngnn
    for gf in (True, False):
        kw = dict(batch_size=256, shuffle=True, seed=11, gather_features=gf)
        ref = list(NeighborLoader(graph, graph.train_idx, [15, 10], **kw))
        sf = NeighborLoader(graph, graph.train_idx, [15, 10], sync_free=True, **kw)
        n_b = 0
        for b, blk in enumerate(sf):
            torch.cuda.synchronize()
            n, E = (int(v) for v in blk.edge_index._ngnn_counts[:2].tolist())
            r = ref[b]
            assert (n, E) == (r.n_id.numel(), r.edge_index.size(1))
            assert torch.equal(blk.n_id[:n], r.n_id) and torch.equal(blk.edge_index[:, :E], r.edge_index)
            assert torch.equal(blk.y[:n], r.y) and blk.batch_size == r.batch_size
            if gf:
                assert torch.equal(blk.x[:n], r.x)
            else:
                assert torch.equal(blk.x.index[:n], r.n_id)
            if b == 0:  # (refused before the capacity-sized rows are touched)
                m = ngnn.SAGE(graph.x.size(1), 16, graph.num_classes, 2).to(DEV)
                with pytest.raises(ValueError, match="sync_free"):
                    m(blk.x, blk.edge_index)
            n_b += 1
        assert n_b == len(ref)
    from ngnn.loader import _sampler_cache
    assert all(bool((st.node_map == -1).all()) for st in _sampler_cache(graph).free)
