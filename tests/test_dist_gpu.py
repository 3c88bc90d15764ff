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


def _worker_headline(rank, world, port, q):
    """the config #4 path -- SAGE(100, 256, 47) (k_fwd2 +
    loss head + k_bwd2 writing the bucket views), products-shaped graph,
    [15, 10] bs 1024 -- through GraphedTrainStep with the split reduce (pack
    in the first graph, one all-reduce, unpack + Adam in the second)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    try:
        import torch.nn.functional as F

        import ngnn
        from ngnn import fused
        from ngnn.distributed import GradAllReduce, init
        from ngnn.graphs import GraphedTrainStep, slot_size
        from ngnn.loader import NeighborLoader, synthetic_graph
        from ngnn.optim import Adam
        import datetime
        import sys
        from test_gpu_configs import _gpu_hidden, _hooked_capture, _slot_masks
        from test_gpu_fused import _MaskedSAGE
        # a short collective timeout: a rank that fails leaves its peer in a
        # collective, which then raises instead of waiting out the test
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=90))
        print(f"[rank {rank}] up", file=sys.stderr, flush=True)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        graph = synthetic_graph("ogbn-products", dev, seed=0, scale=0.03)  # ~2.9 k seeds per rank
        loader = NeighborLoader(graph, graph.train_idx, [15, 10], 1024, shuffle=True, seed=3,
                                rank=rank, world_size=world)
        it = iter(loader)
        warm, b = next(it), next(it)
        torch.manual_seed(1234)
        model = ngnn.SAGE(100, 256, 47, 2, dropout=0.5).to(dev).train()
        init_sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
        opt = Adam(model.parameters(), lr=1e-3)
        red = GradAllReduce(model.parameters())
        n_cap, e_cap = slot_size(1024, [15, 10])
        step = GraphedTrainStep(model, opt, 1024, n_cap, e_cap, 100, dev, reducer=red)
        calls = []
        orig = fused.sage2_backward

        def spy(*a, **k):
            calls.append(1)
            return orig(*a, **k)

        fused.sage2_backward = spy
        try:
            _hooked_capture(step, warm.x, warm.edge_index, warm.y)
        finally:
            fused.sage2_backward = orig
        assert calls, "the captured backward did not take ngnn_sage2_bwd"
        assert step._split_reduce and not step.folded
        print(f"[rank {rank}] captured", file=sys.stderr, flush=True)
        step(b.x, b.edge_index, b.y, b.batch_size)
        torch.cuda.synchronize()
        print(f"[rank {rank}] stepped", file=sys.stderr, flush=True)
        params = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu()
        grads = {k: p.grad.detach().cpu().clone() for k, p in model.named_parameters()}
        # this rank's own gradient, by the oracle on its block with the replay's masks
        seed_state = int(step.seed_state.item()) & (2**64 - 1)
        N = b.num_nodes
        hid, rn = _gpu_hidden(step)
        ref = _MaskedSAGE(100, 256, 47, 2, dropout=0.5, masks=_slot_masks(seed_state, N, 256, 0.5, 2),
                          gpu_hidden=hid, kink_rows=rn)
        ref.load_state_dict(init_sd)
        out_r = ref(b.x.cpu(), b.edge_index.cpu())
        F.cross_entropy(out_r[:b.batch_size], b.y[:b.batch_size].cpu()).backward()
        mine_local = torch.cat([q.grad.reshape(-1) for q in ref.parameters()])
        gathered = [torch.empty_like(mine_local) for _ in range(world)]
        dist.all_gather(gathered, mine_local)
        avg = torch.stack(gathered).mean(0)
        pg = [torch.empty_like(params) for _ in range(world)]
        dist.all_gather(pg, params)
        same_ranks = all(torch.equal(pg[0], t) for t in pg)
        # the single-process step on the rank-averaged oracle gradients
        off, worst, upd = 0, 0.0, 0.0
        for (k, rp) in ref.named_parameters():
            n = rp.numel()
            want = avg[off:off + n].view(rp.shape)
            err = float((grads[k] - want).abs().max()) / max(float(want.abs().max()), 1e-30)
            worst = max(worst, err)
            rp.grad = want.clone()
            off += n
        o_ref = torch.optim.Adam(ref.parameters(), lr=1e-3)
        o_ref.step()
        named = dict(model.named_parameters())
        for k, rp in ref.named_parameters():
            p = named[k].detach().cpu()
            sure = rp.grad.abs() > 1e-2 * rp.grad.abs().max()
            upd = max(upd, float((p[sure] - rp.detach()[sure]).abs().max()))
        q.put((rank, same_ranks, worst, upd, None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put((rank, False, float("inf"), float("inf"), traceback.format_exc()))


@pytest.mark.timeout(300)
def test_headline_model_data_parallel_two_ranks():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_headline, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=150) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
    for rank, same, worst, upd, err in out:
        assert err is None, err
        assert same, f"rank {rank}: parameters differ across ranks"
        # the all-reduced .grad = the mean of the ranks' oracle gradients
        assert worst <= 1e-5, worst
        # and the parameters = torch's Adam step on that mean (step 1: |dp| ~ lr)
        assert upd <= 2e-6, upd
