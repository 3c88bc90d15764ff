"""Seed-sharded data parallelism through the captured HIP-graph step, two
ranks on the one GPU of the test box (gloo carries the CUDA all-reduce here;
the bench uses RCCL, same ngnn.distributed code): the bucket pack / unpack
captured inside the graphs, one all-reduce between the replays.  Checks that
every rank ends with bitwise identical parameters and that the graph step
matches eager training with GradAllReduce on the same batches."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    try:
        import ngnn
        from ngnn.distributed import GradAllReduce, init
        from ngnn.graphs import GraphedTrainStep, slot_size
        from ngnn.loader import NeighborLoader, synthetic_graph
        from ngnn.losses import seed_cross_entropy
        from ngnn.optim import Adam
        init(backend="gloo")
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        graph = synthetic_graph("ogbn-products", dev, seed=0, scale=0.01)
        loader = NeighborLoader(graph, graph.train_idx, [5, 4], 128, shuffle=True, seed=3,
                                rank=rank, world_size=world)
        batches = [b for _, b in zip(range(4), loader)]
        res = {}
        for mode in ("graph", "eager"):
            torch.manual_seed(1234)
            model = ngnn.SAGE(100, 32, 47, 2, dropout=0.0).to(dev).train()
            opt = Adam(model.parameters(), lr=1e-2)
            red = GradAllReduce(model.parameters())
            if mode == "graph":
                n_cap, e_cap = slot_size(128, [5, 4])
                step = GraphedTrainStep(model, opt, 128, n_cap, e_cap, 100, dev, reducer=red)
                step.capture(batches[0].x, batches[0].edge_index, batches[0].y)
                for b in batches:
                    step(b.x, b.edge_index, b.y)
            else:
                for b in batches:
                    out = model(b.x, b.edge_index)
                    loss = seed_cross_entropy(out, b.y, b.batch_size)
                    opt.zero_grad(set_to_none=False)
                    loss.backward()
                    red()
                    opt.step()
            torch.cuda.synchronize()
            res[mode] = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu()
        mine = res["graph"]
        gathered = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(gathered, mine)
        same_ranks = all(torch.equal(gathered[0], g) for g in gathered)
        diff = float((res["graph"] - res["eager"]).abs().max())
        q.put((rank, same_ranks, diff, None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put((rank, False, float("inf"), traceback.format_exc()))


def test_graph_step_data_parallel_two_ranks():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=110) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
    for rank, same, diff, err in out:
        assert err is None, err
        assert same, f"rank {rank}: parameters differ across ranks"
        # graph vs eager: same batches and rule; float-atomic input gradients -> tolerance
        assert diff < 1e-4, diff
