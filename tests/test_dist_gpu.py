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


def _worker_config4(rank, world, port, q):
    """BASELINE config #4's model -- SAGE(100, 256, 256,
    47) in bf16, [20, 15, 10] bs 1024 (config #3's step) -- seed-sharded over
    two ranks through GraphedTrainStep with the split reduce: the bf16
    gradients move into the fp32 bucket and back (divided by the world) by
    ngnn_cast_tensors_ex launches, never an ATen copy."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    try:
        import datetime
        import sys

        import torch.nn.functional as F

        import ngnn
        from ngnn import distributed as ndist
        from ngnn.distributed import GradAllReduce
        from ngnn.graphs import GraphedTrainStep, slot_size
        from ngnn.loader import NeighborLoader, synthetic_graph
        from ngnn.optim import Adam
        from oracle import pyg_ref
        from test_gpu_configs import _hooked_capture, _oracle_rows, _slot_masks
        from test_gpu_fused import dropout_scale
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=120))
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        graph = synthetic_graph("ogbn-products", dev, seed=0, scale=0.03)
        graph.x = graph.x.to(torch.bfloat16)
        loader = NeighborLoader(graph, graph.train_idx, [20, 15, 10], 1024, shuffle=True, seed=5,
                                rank=rank, world_size=world)
        it = iter(loader)
        warm, b = next(it), next(it)
        torch.manual_seed(4321)
        model = ngnn.SAGE(100, 256, 47, 3, dropout=0.5).to(dev).to(torch.bfloat16).train()
        init_sd = {k: v.detach().float().cpu().clone() for k, v in model.state_dict().items()}
        opt = Adam(model.parameters(), lr=1e-3)
        red = GradAllReduce(model.parameters())
        calls = []
        orig_cast, orig_copy = ndist.cast_tensors, torch._foreach_copy_

        def spy(*a, **k):
            calls.append(len(a[0]))
            return orig_cast(*a, **k)

        def no_aten(*a, **k):  # pragma: no cover - the assertion below reports it
            raise AssertionError("torch._foreach_copy_ on the bucket path")

        ndist.cast_tensors, torch._foreach_copy_ = spy, no_aten
        try:
            n_cap, e_cap = slot_size(1024, [20, 15, 10])
            step = GraphedTrainStep(model, opt, 1024, n_cap, e_cap, 100, dev, reducer=red)
            _hooked_capture(step, warm.x, warm.edge_index, warm.y)
            assert step._split_reduce and not step.folded
            step(b.x, b.edge_index, b.y, b.batch_size)
            torch.cuda.synchronize()
        finally:
            ndist.cast_tensors, torch._foreach_copy_ = orig_cast, orig_copy
        assert calls, "the bucket pack / unpack did not take ngnn_cast_tensors_ex"
        print(f"[rank {rank}] stepped", file=sys.stderr, flush=True)
        params = torch.cat([p.detach().float().reshape(-1) for p in model.parameters()]).cpu()
        grads = {k: p.grad.detach().float().cpu().clone() for k, p in model.named_parameters()}
        assert all(p.grad.dtype == torch.bfloat16 for p in model.parameters())
        # this rank's gradient by the oracle (fp32, bf16 storage points), the
        # replay's dropout masks rebuilt from the slot seed
        seed_state = int(step.seed_state.item()) & (2**64 - 1)
        N = b.num_nodes
        masks = _slot_masks(seed_state, N, 256, 0.5, 3)
        ref = pyg_ref.SAGE(100, 256, 47, 3, dropout=0.5)
        ref.load_state_dict(init_sd)
        out_r = _oracle_rows(ref, b.x.float().cpu(), b.edge_index.cpu(), torch.arange(b.batch_size), masks,
                             dropout_scale(0.5), act_dtype=torch.bfloat16)
        F.cross_entropy(out_r, b.y[:b.batch_size].cpu()).backward()
        mine_local = torch.cat([p.grad.reshape(-1) for p in ref.parameters()])
        gathered = [torch.empty_like(mine_local) for _ in range(world)]
        dist.all_gather(gathered, mine_local)
        avg = torch.stack(gathered).mean(0)
        pg = [torch.empty_like(params) for _ in range(world)]
        dist.all_gather(pg, params)
        same_ranks = all(torch.equal(pg[0], t) for t in pg)
        off, worst, where = 0, 0.0, ""
        for k, rp in ref.named_parameters():
            n = rp.numel()
            want = avg[off:off + n].view(rp.shape)
            # config #3's bf16 bar (test_config_products_3layer_bf16_graph_step:
            # |g - g_ref| <= 2e-2 max|g_ref| + 2e-2 |g_ref|) held by each rank's
            # own gradient, so the mean of the ranks' gradients is held to the
            # mean of their bars (the ranks' gradients partly cancel: a bar of
            # the mean's own magnitude would be tighter than either rank's)
            bar = sum(2e-2 * float(gr[off:off + n].abs().max()) + 2e-2 * gr[off:off + n].abs()
                      for gr in gathered).view(rp.shape) / world
            ratio = (grads[k] - want).abs() / bar.clamp_min(1e-30)
            if float(ratio.max()) > worst:
                i = int(ratio.argmax())
                worst = float(ratio.max())
                where = (f"{k}[{i}]: got {float(grads[k].flatten()[i]):.4g} want {float(want.flatten()[i]):.4g} "
                         f"bar {float(bar.flatten()[i]):.3g}")
            off += n
        q.put((rank, same_ranks, (worst, where), None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put((rank, False, (float("inf"), ""), traceback.format_exc()))


@pytest.mark.timeout(400)
def test_config4_bf16_3layer_data_parallel_two_ranks():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_config4, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
    for rank, same, worst, err in out:
        assert err is None, err
        assert same, f"rank {rank}: parameters differ across ranks"
        # the all-reduced bf16 .grad = the mean of the ranks' oracle gradients
        # at the SURVEY 8(c) bf16 bar (the ratio to the bar: <= 1)
        assert worst[0] <= 1.0, worst


def _worker_rccl(port, q):
    """The RCCL backend on this box's one GPU: a world-1 "nccl" process group
    (RCCL refuses two ranks on one device), the bucket's pack, the RCCL
    all_reduce -- eager and captured in a HIP graph -- and unpack, through
    ngnn.distributed as the bench's N-GPU run takes them."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    try:
        import datetime

        import ngnn
        from ngnn.distributed import GradAllReduce
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev,
                                timeout=datetime.timedelta(seconds=90))
        assert dist.get_backend() == "nccl"
        torch.manual_seed(0)
        model = ngnn.SAGE(100, 256, 47, 2).to(dev)
        red = GradAllReduce(model.parameters())
        want = []
        for p in model.parameters():
            p.grad = torch.randn_like(p)
            want.append(p.grad.detach().clone())
        red.pack()
        red.allreduce()
        red.unpack()
        torch.cuda.synchronize()
        err = max(float((p.grad - w).abs().max()) for p, w in zip(model.parameters(), want))
        # the all-reduce captured in a graph (the split reduce's collective
        # is eager; this checks RCCL's capture on the bucket too)
        red.bucket.fill_(1.0)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            red.allreduce()  # (warm-up on the side stream)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            red.allreduce()
        g.replay()
        torch.cuda.synchronize()
        ok_graph = bool(torch.all(red.bucket == 1.0))
        q.put((err, ok_graph, None))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put((float("inf"), False, traceback.format_exc()))


@pytest.mark.timeout(200)
def test_rccl_backend_world1_bucket_allreduce():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker_rccl, args=(_free_port(), q))
    p.start()
    err, ok_graph, tb = q.get(timeout=150)
    p.join(timeout=30)
    assert tb is None, tb
    assert err == 0.0, err  # (one rank: the sum is the rank's own bucket, / 1 exact)
    assert ok_graph
