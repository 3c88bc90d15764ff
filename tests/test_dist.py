"""Seed-node data parallelism on CPU with the gloo backend, world_size 2.

Checks the two pieces of ngnn.distributed the GPU path uses unchanged:
shard_seeds (same permutation on every rank, disjoint strided slices) and
GradAllReduce (one flat bucket, SUM / world).  The model here is the oracle
SAGE on CPU (the product kernels need a GPU); the all-reduce logic is
device-agnostic.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, dtype="f32"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        from ngnn.distributed import GradAllReduce, init, shard_seeds
        from oracle import pyg_ref
        r, w, _ = init(backend="gloo")
        assert (r, w) == (rank, world)
        # sharding
        nodes = torch.arange(1000)
        mine = shard_seeds(nodes, rank, world, epoch=3, seed=11)
        gathered = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(gathered, mine)
        allseeds = torch.cat(gathered)
        ok_shard = bool(torch.equal(allseeds.sort().values, nodes))
        # gradient all-reduce == mean of per-rank gradients
        torch.manual_seed(0)
        model = pyg_ref.SAGE(6, 8, 3, 2, dropout=0.0)
        if dtype == "bf16":  # BASELINE config #3's model dtype
            model = model.to(torch.bfloat16)
        elif dtype == "mixed":  # bf16 and fp32 parameters in one bucket
            model.convs[0].to(torch.bfloat16)
        g = torch.Generator().manual_seed(100)
        data = [(torch.randn(20, 6, generator=g), torch.randint(0, 20, (2, 60), generator=g),
                 torch.randint(0, 3, (20,), generator=g)) for _ in range(world)]
        local_grads = []
        def fwd(x, ei):
            if dtype == "f32":
                return model(x, ei)
            h = model.convs[0](x.to(model.convs[0].lin_l.weight.dtype), ei).relu()
            return model.convs[1](h.to(model.convs[1].lin_l.weight.dtype), ei).float()
        for (x, ei, y) in data:
            model.zero_grad()
            torch.nn.functional.cross_entropy(fwd(x, ei)[:5], y[:5]).backward()
            local_grads.append([p.grad.clone() for p in model.parameters()])
        # the bucket's arithmetic: widen, sum in fp32, / world, round to the parameter dtype
        want = [(sum(g.float() for g in gs) / world).to(gs[0].dtype) for gs in zip(*local_grads)]
        model.zero_grad()
        x, ei, y = data[rank]
        torch.nn.functional.cross_entropy(fwd(x, ei)[:5], y[:5]).backward()
        GradAllReduce(model.parameters())()
        ok_grad = all(p.grad.dtype == w_.dtype and torch.allclose(p.grad.float(), w_.float(), atol=1e-6)
                      for p, w_ in zip(model.parameters(), want))
        q.put((rank, ok_shard, ok_grad, mine.numel()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported through the queue
        q.put((rank, False, False, repr(e)))


@pytest.mark.timeout(120)
@pytest.mark.parametrize("dtype", ["f32", "bf16", "mixed"])
def test_gloo_world2_sharding_and_grad_allreduce(dtype):
    """f32, a bf16 model (BASELINE config #3 under data parallelism) and a
    mixed one: the bf16 gradients go through the fp32 bucket (one
    multi-tensor copy each way) and come back rounded to bf16."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, dtype)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=30)
    res.sort()
    assert all(r[1] for r in res), res
    assert all(r[2] for r in res), res
    assert sum(r[3] for r in res) == 1000


def test_shard_seeds_single_process():
    from ngnn.distributed import shard_len, shard_seeds
    nodes = torch.arange(10)
    a = shard_seeds(nodes, 0, 3, epoch=0, seed=1)
    b = shard_seeds(nodes, 1, 3, epoch=0, seed=1)
    c = shard_seeds(nodes, 2, 3, epoch=0, seed=1)
    # equal shards (10 seeds over 3 ranks: padded cyclically to 12), covering every seed
    assert a.numel() == b.numel() == c.numel() == shard_len(10, 3) == 4
    assert torch.equal(torch.cat([a, b, c]).unique(), nodes)
    assert torch.equal(shard_seeds(nodes, 0, 1, epoch=0, seed=1).sort().values, nodes)
    assert not torch.equal(shard_seeds(nodes, 0, 1, epoch=0, seed=1),
                           shard_seeds(nodes, 0, 1, epoch=1, seed=1))


def _loader_worker(rank, world, port, q, n_seeds, bs):
    """Every rank iterates its NeighborLoader shard's batch count and joins one
    all-reduce per batch (the data-parallel step's collective), then a barrier:
    unequal batch counts would leave some ranks in an all-reduce the others
    never join (caught by the timeouts)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        import datetime
        from ngnn.loader import Graph, NeighborLoader
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=60))
        g = Graph(torch.zeros(n_seeds + 1, dtype=torch.int64), torch.zeros(0, dtype=torch.int32),
                  torch.zeros(n_seeds, 4), torch.zeros(n_seeds, dtype=torch.int64),
                  torch.arange(n_seeds), 2)
        loader = NeighborLoader(g, g.train_idx, [2], bs, shuffle=True, seed=3, rank=rank,
                                world_size=world)
        seeds = loader._seeds()
        n_batches = len(loader)
        t = torch.zeros(1)
        for _ in range(n_batches):
            dist.all_reduce(t)
        counts = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(counts, torch.tensor([n_batches, seeds.numel()]))
        allseeds = [torch.empty_like(seeds) for _ in range(world)]
        dist.all_gather(allseeds, seeds)
        covered = bool(torch.equal(torch.cat(allseeds).unique(), torch.arange(n_seeds)))
        dist.barrier()
        q.put((rank, [tuple(c.tolist()) for c in counts], covered))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported through the queue
        q.put((rank, repr(e), False))


@pytest.mark.timeout(180)
def test_gloo_world8_equal_batch_counts():
    """196,615 products seeds over 8 ranks would give rank 7 one
    batch fewer at bs 1024 (24,577 vs 24,576 seeds).  Same arithmetic here:
    n % world != 0 and the per-rank counts straddle a batch boundary."""
    world, bs = 8, 4
    n = 8 * 4 * 3 + 7  # ranks 0-6 would get 13 seeds (4 batches), rank 7 12 (3 batches)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_loader_worker, args=(r, world, port, q, n, bs)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=150) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    for r in res:
        assert isinstance(r[1], list), r
        assert r[2], r
    counts = res[0][1]
    assert len(set(counts)) == 1, counts  # same (batches, seeds) on every rank
    assert counts[0] == (4, 13)
