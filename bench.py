"""Headline benchmark: aggregated edges/s (+ epoch time) of GraphSAGE training
on ogbn-products-shaped mini-batches, fanout [15,10], batch 1024 (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W]   (N > 1: starts N ranks itself)
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

Workload (config.workload = "products-[15,10]-bs1024"): synthetic graph with
ogbn-products' published sizes (N=2,449,029, 123.7 M directed entries, F=100,
C=47, 196,615 train seeds; datasets cannot be downloaded here), model
SAGE(100, 256, 47, num_layers=2, dropout=0.5) + Adam(1e-3), fp32 — the
reference's PipelineCO baseline loop (pipeline.py:152-169).

A "step" = one training iteration over one mini-batch already resident in HBM
(sampled on the GPU before the timed region): forward of both SAGE layers over
the whole block, cross-entropy on the seed rows, backward, RCCL gradient
all-reduce (N>1) and Adam.  Aggregated edges per step = num_layers x E_batch
(every layer aggregates all E edges of the block, sage.py:33-34).
value = sum over ranks of edges / max-over-ranks wall time.

Also reported: epoch_time_s — one full pass over this rank's train seeds
INCLUDING GPU sampling + feature gather (193 batches at N=1); graph mode: the
sync-free loader (no host wait per batch) with the fused x[n_id] gather
(epoch_mode), beside it the sync-free loader with the loader's row copy and
the synchronous loader (one event wait per batch); the roofline
of the dominant kernel (HIP events around every launch inside the timed
region); the reference-equivalent CPU path timed on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "noise-gnn_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
MFMA_F32_PEAK_TFS = 157.3  # dense fp32 MFMA (v_mfma_f32_*_f32), same table


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch-size", type=int, default=1024)
    ap.add_argument("--fanout", type=str, default="15,10")
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--num-layers", type=int, default=0,
                    help="model layers (default: one per fanout hop; config_arxiv5.yml runs 3 layers "
                         "over a [10,5] block -- every layer aggregates all of the block's edges)")
    ap.add_argument("--scale", type=float, default=1.0, help="graph size scale (tests)")
    ap.add_argument("--dataset", default="ogbn-products",
                    help="synthetic graph shape (ngnn.loader.DATASETS); the headline is ogbn-products")
    ap.add_argument("--aggr", default="mean", choices=["mean", "max", "sum"])
    ap.add_argument("--module", default="sage", choices=["sage", "gcn"],
                    help="model.py's `module`: SAGE (sage.py) or SimpleGCN (convolution.py)")
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"],
                    help="model / feature storage dtype (bf16: bf16 feature rows and one-part bf16 weight images, fp32 accumulation)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-epoch", action="store_true")
    ap.add_argument("--no-eager-ref", action="store_true",
                    help="skip the eager reference-loop timing (eager_drop_in)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--eager", action="store_true",
                    help="launch every kernel from Python instead of replaying the captured "
                         "HIP graph of the step")
    ap.add_argument("--gather", default="loader", choices=["fused", "loader"],
                    help="loader (default): the sampler copies x[n_id] into each batch, as "
                         "the reference's loader does (pipeline.py:153); fused: batches carry "
                         "x = graph.x[n_id] unmaterialized and the layer-0 kernels gather the "
                         "rows (graph replay) -- no copy in the loader, +6 us L0 forward and "
                         "+5 us L0 weight gradient in the step (scattered 400-B row reads)")
    ap.add_argument("--coteaching", action="store_true",
                    help="the co-teaching step instead (pipeline.py:95-142, config_products.yml "
                         "algo_type 'coteaching'): two SAGE models, CTLoss, both backwards and Adam "
                         "steps as one graph replay (ngnn.graphs.GraphedCoTeachingStep); noisy labels "
                         "--noise-rate, forget rate --forget-rate; aggregated edges count both models")
    ap.add_argument("--forget-rate", type=float, default=0.36,
                    help="co-teaching forget rate (config_products.yml: noise_rate 0.3 x ct_tau 1.2)")
    ap.add_argument("--noise-rate", type=float, default=0.3)
    ap.add_argument("--timer", default="sage_fwd_l0,sage_fwd_l1,gcn_fwd_l1_z,gcn_fwd_l1_agg,"
                                       "sage2_edge,sage2_fwd,sage2_narrow",
                    help="comma list of kernel spans timed with HIP events in the timed region "
                         "('all', or 'none' for profiler runs)")
    return ap.parse_args()


def pmc_traffic(span, workload, dtype):
    """HBM bytes per launch of the kernel behind `span` ON THIS WORKLOAD AND
    DTYPE from the committed PMC summary (tools/gpu_pmc.sh +
    tools/pmc_traffic.py: FETCH_SIZE x 2 on gfx950 plus WRITE_SIZE, separate
    passes; records keyed "span|workload|dtype"), or (None, None) when that
    combination was never profiled -- never another workload's number."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            rec = json.load(f).get(f"{span}|{workload}|{dtype}")
    except (OSError, ValueError):
        return None, None
    if not rec:
        return None, None
    return int(rec["traffic_bytes"]), f"profiles/pmc_traffic.json ({rec.get('source', '?')})"


def _rows(x):
    """A batch's feature rows as a tensor (IndexedRows: gathered here)."""
    return x.materialize() if hasattr(x, "materialize") else x


def train_step(model, opt, reducer, b):
    from ngnn.losses import seed_cross_entropy  # == F.cross_entropy(out[:bs], y[:bs])
    out = model(b.x, b.edge_index)
    loss = seed_cross_entropy(out, b.y, b.batch_size)
    opt.zero_grad(set_to_none=False)  # keep the grad tensors (a captured graph owns them)
    loss.backward()
    reducer()
    opt.step()
    return loss


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_threads() -> int:
    """Every CPU this process may run on: the affinity mask (the GPU box gives
    each GPU's job a share of the host, OMP_NUM_THREADS = that share), capped
    by os.cpu_count()."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(n, 1)


def cpu_baseline(batches, args, layers):
    """The reference's CPU path: the PyG 2.5.1 op sequence restated in torch
    (oracle/pyg_ref.py), full training steps (fwd + bwd + Adam) over the
    bench's own sampled blocks of the same workload (cycled), for about
    args.cpu_seconds at every available thread, then a bounded 1-thread run
    (all cores and 1 thread, CPU model named)."""
    from oracle import pyg_ref
    from ngnn.loader import DATASETS
    _, _, F_in, C, _ = DATASETS[args.dataset]
    host = [(_rows(b.x).cpu(), b.edge_index.cpu(), b.y.cpu(), b.batch_size) for b in batches]

    def run(threads, seconds, max_steps):
        torch.set_num_threads(threads)
        torch.manual_seed(0)
        m = (pyg_ref.SimpleGCN(F_in, args.hidden, C, layers, dropout=0.5) if args.module == "gcn"
             else pyg_ref.SAGE(F_in, args.hidden, C, layers, dropout=0.5, aggr=args.aggr))
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        x, ei, y, bs = host[0]
        pyg_ref.train_step(m, opt, x, ei, y, bs)  # warm
        n, edges, t0 = 0, 0, time.perf_counter()
        while True:
            x, ei, y, bs = host[n % len(host)]
            pyg_ref.train_step(m, opt, x, ei, y, bs)
            n += 1
            edges += layers * ei.shape[1]
            dt = time.perf_counter() - t0
            if dt >= seconds or n >= max_steps:
                break
        return edges / dt, 1e3 * dt / n, n

    threads0 = torch.get_num_threads()
    threads = _cpu_threads()
    rate, ms, n = run(threads, args.cpu_seconds, 50)
    rate1, ms1, n1 = run(1, max(args.cpu_seconds / 3, 1.0), 3)
    torch.set_num_threads(threads0)
    E = sum(ei.shape[1] for _, ei, _, _ in host[:n]) / min(n, len(host))
    return {"value": rate, "unit": "edges/s", "cores": threads, "kind": "port",
            "ms_per_step": ms, "cpu_model": _cpu_model(), "host_cpus": os.cpu_count(),
            "single_thread": {"value": rate1, "unit": "edges/s", "ms_per_step": ms1, "steps": n1},
            "sample": f"{n} training steps (fwd+bwd+Adam) over {min(n, len(host))} sampled "
                      f"{args.dataset}-[{args.fanout}] bs={args.batch_size} blocks "
                      f"(avg E={E:.0f}) at {threads} threads, then {n1} at 1 thread; "
                      f"torch {torch.__version__} CPU; PyG 2.5.1 op sequence restated in "
                      f"oracle/pyg_ref.py"}


def _eager_node_loaded() -> bool:
    """Did the eager loop run the stack's C++ autograd node (ngnn_eager.so)?"""
    from ngnn import _eager, fused
    return _eager.load() is not None and fused.eager_ext_calls > 0


def eager_reference_loop(batches, args, F_in, C, layers, dev, steps, verbatim=False, ngnn_adam=False):
    """The reference's training loop (pipeline.py:152-169) run verbatim on
    ngnn's modules after the INTEGRATION.md Option-B swap -- no graph capture,
    no loss head, no Adam fold: out = model(x, edge_index)[:batch_size];
    F.cross_entropy; optimizer.zero_grad(); loss.backward(); and the
    reference optimiser, torch.optim.Adam (model.py:66-69).  verbatim: also
    the loop's per-step host reads (total_loss += float(loss), the
    accuracy count).  Returns ms per step over `steps` batches."""
    import torch.nn.functional as F

    import ngnn
    torch.manual_seed(1234)
    if args.module == "gcn":
        model = ngnn.SimpleGCN(F_in, args.hidden, C, layers, dropout=0.5).to(dev)
    else:
        model = ngnn.SAGE(F_in, args.hidden, C, layers, dropout=0.5, aggr=args.aggr).to(dev)
    if args.dtype == "bf16":
        model = model.to(torch.bfloat16)
    # (ngnn_adam: the optimizer swapped too -- ngnn.optim.Adam, the same
    # constructor, one device launch per step)
    from ngnn.optim import Adam as NgnnAdam
    opt = (NgnnAdam if ngnn_adam else torch.optim.Adam)(model.parameters(), lr=1e-3)
    model.train()
    total_loss, total_correct = 0.0, 0

    def one(b):
        nonlocal total_loss, total_correct
        out = model(_rows(b.x), b.edge_index)[:b.batch_size]
        y = b.y[:b.batch_size].squeeze()
        loss = F.cross_entropy(out, y)
        if verbatim:
            total_loss += float(loss)
            total_correct += int(out.argmax(dim=-1).eq(y).sum())
        opt.zero_grad()
        loss.backward()
        opt.step()

    for i in range(3):
        one(batches[i % len(batches)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        one(batches[i % len(batches)])
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / steps


def l0_launch_us(gstep, model, aggr: str, timed, flush_mb: int = 512, dom: str = "sage_fwd_l0"):
    """Per-launch duration of the captured step's layer-0 kernel, measured
    with HIP events on the stream it runs on (events cannot be recorded
    inside the step's own graph on ROCm).  The launch is captured alone into a
    graph over the slot; for EVERY timed batch the slot is loaded exactly as
    the step loads it and that graph replayed between two events:

    * "step"  -- right after the batch's slot load, as inside the step (the
      batch's rows were sampled before the timed region: not cache-resident);
    * "cold"  -- the same after writing a flush_mb buffer, so neither the
      4 MiB L2s nor the 256 MiB MALL hold any of its input;
    * "warm"  -- an immediate second replay on the same batch (its rows now
      partly MALL-resident: the round-2 figure's condition).

    Returns {condition: mean us over the batches}; each figure includes the
    dispatch gap between an event and the kernel (about 1-2 us).

    dom "sage2_fwd": the two-layer forward's main launch (k_fwd2); its
    predecessors in the step (weight images, the edge rows' aggregate + nb)
    run right before it in every graph, and the "seq" figure subtracts a
    graph that holds them too."""
    from ngnn import _lib, fused
    from ngnn.block import get_block
    blk = get_block(gstep.ei, gstep.n_cap)
    c = model.convs[0]
    x = gstep.x
    p = model.dropout if model.training else 0.0
    pre = None
    if dom == "sage2_fwd":
        # (SimpleGCN: [W, b, None] per conv -- the two-layer kernels with W_r = 0)
        params = fused.sage2_params(
            [q.detach() if q is not None else None for cv in model.convs
             for q in ((cv.lin_l.weight, cv.lin_l.bias, cv.lin_r.weight) if hasattr(cv, "lin_l")
                       else (cv.lin.weight, cv.bias, None))])
        root0 = hasattr(c, "lin_l")  # (SimpleGCN: no root term, x never read)
        bufs = fused.sage2_forward(x, blk, aggr, params, p, 0, blk.seed_dev, root0=root0)
        # (fused: the edge and main phases are one launch, k_fwd2x -- timed
        # together, as the step runs them)
        fz = fused.fwd2_fused()

        def pre():
            fused.sage2_forward(x, blk, aggr, params, p, 0, blk.seed_dev,
                                stages=_lib.SAGE2_PREP | (0 if fz else _lib.SAGE2_EDGE), bufs=bufs, root0=root0)

        def run():
            fused.sage2_forward(x, blk, aggr, params, p, 0, blk.seed_dev,
                                stages=_lib.SAGE2_MAIN | (_lib.SAGE2_EDGE if fz else 0), bufs=bufs, root0=root0)
    else:
        wl, bl, wr = (q.detach().float() for q in (c.lin_l.weight, c.lin_l.bias, c.lin_r.weight))
        agg = fused.agg_buffer(gstep.n_cap, x.size(1), x.device, wl.shape[0])
        w1 = c.lin_l.weight.dtype == torch.bfloat16

        def run():
            fused.sage_layer_fwd(x, blk, aggr, wl, bl, wr, relu=True, p_drop=p, seed=0, agg_out=agg,
                                 seed_dev=blk.seed_dev, x_dev=blk.x_dev, xrow_dev=blk.xrow_dev,
                                 x_rows=blk.x_rows, w_bf16=w1)
    if pre is not None:
        pre()
    run()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        run()
    gpre = None
    if pre is not None:
        gpre = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gpre):
            pre()
    res = {"seq": [], "step": [], "cold": [], "warm": []}
    # "seq" -- the in-step figure: R timed batches as ONE graph of [slot load,
    # layer-0 launch] pairs minus a graph of the R slot loads alone, divided by
    # R (each launch right after its batch's slot load, back to back as in the
    # step; no event sits next to a single launch)
    R = min(len(timed), 20)
    try:
        gs = []
        for with_l0 in (True, False):
            gg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gg):
                for b in timed[:R]:
                    gstep.load(b.x, b.edge_index, b.y, zero_copy=gstep.zero_copy,
                               batch_size=b.batch_size)
                    if pre is not None:
                        pre()
                    if with_l0:
                        run()
            gs.append(gg)
        tt = {0: [], 1: []}
        for _ in range(3):
            for i, gg in enumerate(gs):
                gg.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                gg.replay()
                e1.record()
                e1.synchronize()
                tt[i].append(e0.elapsed_time(e1) * 1e3)
        res["seq"].append((sorted(tt[0])[1] - sorted(tt[1])[1]) / R)
        del gs
    except RuntimeError as e:  # a capture this build refuses: the per-launch figures only
        res["seq"] = []
        print(f"[bench] in-step sequence timing unavailable: {e}", file=sys.stderr)
    flush = torch.empty(flush_mb << 20, dtype=torch.uint8, device=x.device)
    hrows = []
    for b in timed:
        for cond in ("step", "cold"):  # (step first: the cold run leaves the rows resident)
            gstep.load(b.x, b.edge_index, b.y, zero_copy=gstep.zero_copy, batch_size=b.batch_size)
            if cond == "step":  # the rows of h the step writes: the slot's R' (low word)
                hrows.append(min(int(gstep.r_next.item()) & 0xFFFFFFFF, b.num_nodes))
            if gpre is not None:
                gpre.replay()
            if cond == "cold":
                flush.fill_(cond == "cold")
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            evs[0].record()
            g.replay()
            evs[1].record()
            if cond == "step":
                evs[2].record()
                g.replay()
                evs[3].record()
            (evs[3] if cond == "step" else evs[1]).synchronize()
            res[cond].append(evs[0].elapsed_time(evs[1]) * 1e3)
            if cond == "step":
                res["warm"].append(evs[2].elapsed_time(evs[3]) * 1e3)
    del flush
    out = {k: sum(v) / len(v) for k, v in res.items() if v}
    out["hrows"] = hrows
    return out


def _allreduce_name(world: int) -> str:
    """Which collective carries the gradient all-reduce (gloo only in rehearsals)."""
    import torch.distributed as dist
    if world <= 1 or not dist.is_initialized():
        return "RCCL"
    return "RCCL" if dist.get_backend() == "nccl" else dist.get_backend()


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """`python bench.py --gpus N` without torchrun's env: start the N ranks
    here, one child process per GPU with RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* set (what torchrun would set), and return the first non-zero
    exit code.  This process never touches the GPU (no exec after a HIP
    call: children only)."""
    import subprocess
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        print(f"[bench] rank exit codes {rcs}", file=sys.stderr)
    return bad[0] if bad else 0


def check_world(gpus: int, world: int) -> None:
    """The run must have exactly --gpus ranks, one per GPU (a mismatch would
    print a line whose n_gpus is not what was asked for)."""
    if world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but the process group has {world} rank(s) "
                         f"(WORLD_SIZE={os.environ.get('WORLD_SIZE')}); launch with "
                         f"torchrun --nproc-per-node {gpus} or without torchrun's env")
    rehearsal = os.environ.get("NGNN_DIST_BACKEND") == "gloo"
    if world > 1 and not rehearsal and torch.cuda.device_count() < world:
        raise SystemExit(f"bench.py: --gpus {world} needs {world} visible GPUs, found "
                         f"{torch.cuda.device_count()} (NGNN_DIST_BACKEND=gloo rehearses "
                         f"several ranks on fewer GPUs)")


def allreduce_us(reducer, world: int, reps: int = 50):
    """Host-timed gradient all-reduce of the step's bucket (the one
    collective of a DP step), averaged over `reps` calls between syncs."""
    if world <= 1 or not reducer.active():
        return None
    import torch.distributed as dist
    saved = reducer.bucket.clone()
    for _ in range(5):
        reducer.allreduce()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        reducer.allreduce()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    reducer.bucket.copy_(saved)
    t = torch.tensor([dt], dtype=torch.float64, device=reducer.bucket.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return {"us": round(1e6 * float(t), 2), "bytes": reducer.bucket.numel() * 4, "reps": reps,
            "note": "host-timed all_reduce(SUM) of the flat fp32 gradient bucket, max over ranks"}


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    import torch.distributed as dist

    import ngnn
    from ngnn import _timing
    from ngnn.distributed import GradAllReduce, init
    from ngnn.loader import NeighborLoader, sample_block, synthetic_graph

    rank, world, local = init()
    check_world(args.gpus, world)
    # (one GPU per rank; modulo only matters when rehearsing N ranks on fewer GPUs)
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    fanout = [int(v) for v in args.fanout.split(",")]
    layers = args.num_layers or len(fanout)

    from ngnn.loader import DATASETS
    _, _, F_in, C, _ = DATASETS[args.dataset]
    graph = synthetic_graph(args.dataset, dev, seed=0, scale=args.scale)
    torch.manual_seed(1234)  # identical init on every rank
    if args.module == "gcn":
        model = ngnn.SimpleGCN(F_in, args.hidden, C, layers, dropout=0.5).to(dev)
    else:
        model = ngnn.SAGE(F_in, args.hidden, C, layers, dropout=0.5, aggr=args.aggr).to(dev)
    if args.dtype == "bf16":
        model = model.to(torch.bfloat16)
        graph.x = graph.x.to(torch.bfloat16)
    # the reference's Adam(lr=1e-3) rule as ngnn's two-launch device Adam; its step count
    # lives on the device, so the HIP graph can replay it
    from ngnn.optim import Adam
    opt = Adam(model.parameters(), lr=1e-3)
    reducer = GradAllReduce(model.parameters())
    model.train()
    ct = None
    if args.coteaching:
        # config_products.yml's train_ct: a second model, noisy labels (30 % flipped
        # uniformly, flip_label's role), CTLoss at the steady forget rate
        if world > 1 or args.eager:
            raise SystemExit("bench.py --coteaching: one GPU, graph replay")
        from ngnn.losses import CTLoss
        model2 = ngnn.SAGE(F_in, args.hidden, C, layers, dropout=0.5, aggr=args.aggr).to(dev)
        if args.dtype == "bf16":
            raise SystemExit("bench.py --coteaching: fp32 (CTLoss takes fp32 logits)")
        model2.train()
        opt2 = Adam(model2.parameters(), lr=1e-3)
        gen = torch.Generator(device=dev).manual_seed(17)
        flip = torch.rand(graph.num_nodes, device=dev, generator=gen) < args.noise_rate
        yhn = torch.where(flip, torch.randint(0, C, (graph.num_nodes,), device=dev, generator=gen), graph.y)
        graph.node_attrs["yhn"] = yhn  # batch.yhn, gathered by the loader (pipeline.py:116)
        ct = (model2, opt2, CTLoss(dev), yhn == graph.y)

    # pre-sample this rank's batches (inputs resident in HBM before timing)
    loader = NeighborLoader(graph, graph.train_idx, fanout, args.batch_size, shuffle=True, seed=7,
                            rank=rank, world_size=world, gather_features=args.gather == "loader")
    it = iter(loader)
    nb = min(len(loader), args.steps + args.warmup)
    batches = [next(it) for _ in range(nb)]
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    graph_data = graph  # (the name `graph` is the replay switch below)
    graph = not args.eager
    if ct is not None:
        from ngnn.graphs import GraphedCoTeachingStep, slot_size
        n_cap, e_cap = slot_size(args.batch_size, fanout)
        gstep = GraphedCoTeachingStep(model, opt, ct[0], ct[1], ct[2], args.batch_size, n_cap, e_cap,
                                      batches[0].x.size(1), dev, noise_or_not=ct[3])
        b0 = batches[0]
        gstep.capture(b0.x, b0.edge_index, b0.yhn, b0.n_id, args.forget_rate)

        def run(b):
            gstep(b.x, b.edge_index, b.yhn, b.n_id, args.forget_rate, b.batch_size)
    elif graph:
        # the whole step (CSR build .. Adam) as one captured HIP graph over a
        # static slot sized for any block of this fanout (ngnn/graphs.py)
        from ngnn.graphs import GraphedTrainStep, slot_size
        n_cap, e_cap = slot_size(args.batch_size, fanout)
        gstep = GraphedTrainStep(model, opt, args.batch_size, n_cap, e_cap, batches[0].x.size(1), dev,
                                 reducer=reducer)
        gstep.capture(batches[0].x, batches[0].edge_index, batches[0].y)

        def run(b):
            gstep(b.x, b.edge_index, b.y, b.batch_size)
    else:
        def run(b):
            train_step(model, opt, reducer, b)

    for i in range(args.warmup):
        run(batches[i % nb])
    barrier()
    timer_names = None if args.timer == "all" else ([] if args.timer == "none" else args.timer.split(","))

    def new_timer():
        t = _timing.KernelTimer(only=None if args.timer == "all" else (timer_names or ["-"]))
        t.reserve(8 * args.steps if args.timer != "none" else 0)
        return t
    # eager: per-launch events inside the timed region; graph: events cannot be
    # recorded inside a captured graph on ROCm, so the same kernels on the same
    # batches are timed in an eager pass right after the timed replays
    timer = new_timer() if not graph else _timing.KernelTimer(only=["-"])
    edges = 0
    t0 = time.perf_counter()
    with timer:
        for i in range(args.steps):
            b = batches[(args.warmup + i) % nb]
            run(b)
            edges += (2 if ct is not None else 1) * layers * b.edge_index.shape[1]
    t_issue = time.perf_counter() - t0  # host time to enqueue the K steps
    barrier()
    dt = time.perf_counter() - t0
    if graph and args.timer != "none" and ct is None:
        timer = new_timer()
        with timer:
            for i in range(args.steps):
                train_step(model, opt, reducer, batches[(args.warmup + i) % nb])
        barrier()
    ar = allreduce_us(reducer, world)
    t = torch.tensor([dt, float(edges)], dtype=torch.float64, device=dev)
    if world > 1:
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        dt, edges = float(tmax[0]), float(t[1])
    else:
        dt, edges = float(t[0]), float(t[1])

    workload = f"{args.dataset.replace('ogbn-', '')}-[{args.fanout}]-bs{args.batch_size}"
    if layers != len(fanout):
        workload += f"-L{layers}"
    if args.aggr != "mean" and args.module == "sage":
        workload += f"-{args.aggr}"
    if args.module == "gcn":
        workload += "-gcn"
    if ct is not None:
        workload += f"-coteaching-fr{args.forget_rate:g}"
    # the layer-0 kernel reads rows through n_id under the fused gather: its
    # own traffic key (a loader-copy PMC record is not its evidence)
    pmc_workload = workload + ("-fusedgather" if args.gather == "fused" else "")
    # dominant kernel roofline from the live events of the timed region
    summ = timer.summary()
    dom = max(summ.items(), key=lambda kv: kv[1][1]) if summ else None
    roof = None
    l0 = eager_us = None
    if dom:
        name, (n, ms, nbytes, flops, mfma_s) = dom
        eager_us = 1e3 * ms / n
        if graph and (name == "sage2_fwd" or (name == "sage_fwd_l0" and args.module == "sage")):
            # the same kernel on the same timed batches, each right after its
            # slot load (see l0_launch_us); algorithmic bytes / flops per
            # launch from the eager records of those batches
            timed = [batches[(args.warmup + i) % nb] for i in range(args.steps)]
            l0 = l0_launch_us(gstep, model, "sum" if args.module == "gcn" else args.aggr, timed, dom=name)
            ms = l0.get("seq", l0["step"]) * 1e-3 * n
            if name == "sage2_fwd":
                # in the step h is written only below the slot's R' (the eager
                # pass writes every row): the in-step algorithmic bytes
                nbytes -= sum(4 * 256 * (bb.num_nodes - r) for bb, r in zip(timed, l0["hrows"]))
        t = ms * 1e-3
        gbs = nbytes / t / 1e9
        tfs = flops / t / 1e12
        # the binding roof is the larger ideal time: HBM bytes at 8 TB/s, or
        # the matrix-core time of the launch's instruction mix (the root term
        # runs 6 bf16 MFMA products per f32 product: its f32-equivalent peak is
        # flops / mfma_s, 2.7x the f32 MFMA peak; exact mode: the f32 peak)
        t_hbm = nbytes / (HBM_PEAK_GBS * 1e9)
        f_hbm, f_mfma = t_hbm / t, mfma_s / t
        mfma_peak = flops / mfma_s / 1e12 if mfma_s > 0 else MFMA_F32_PEAK_TFS
        if mfma_s > t_hbm:
            roof = {"kernel": name, "bound": "mfma", "achieved": round(tfs, 2),
                    "peak": round(mfma_peak, 1), "unit": "TFLOP/s", "frac": round(f_mfma, 4)}
        else:
            roof = {"kernel": name, "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(f_hbm, 4)}
        traffic, traffic_src = pmc_traffic(name, pmc_workload, args.dtype)
        roof.update({
            "traffic": traffic, "traffic_src": traffic_src, "launches": n,
            "avg_us": round(1e3 * ms / n, 2),
            "timed_in": "timed region (eager)" if not graph else (
                "in-step sequence: HIP events around one replay of a graph of 20 timed batches' "
                "[slot load, layer-0 forward] pairs minus one of the 20 slot loads alone, / 20 "
                "(each launch right after its batch's slot load, back to back, as in the step: "
                "compare rocprof's in-step average of the layer-0 kernels); alg. bytes/flops per "
                "launch from an eager pass over the same batches" if (l0 and "seq" in l0) else
                "HIP events around a graph replay of this one launch on each timed batch, right "
                "after that batch's slot load (as in the step), over all timed batches after the "
                "timed region; alg. bytes/flops per launch from an eager pass over the same "
                "batches" if l0 is not None else
                "eager pass over the timed batches, right after the graph replays"),
            "avg_us_single": None if l0 is None else round(l0["step"], 2),
            "avg_us_cold": None if l0 is None else round(l0["cold"], 2),
            "avg_us_warm": None if l0 is None else round(l0["warm"], 2),
            "cold_warm_note": None if l0 is None else (
                "avg_us: the in-step sequence (timed_in); single: events around one replay of "
                "the launch alone right after its slot load (includes the graph-launch gap); "
                "cold: the same after a 512 MiB write (L2 and MALL hold none of the input); "
                "warm: an immediate second launch on the same batch (partly MALL-resident)"),
            "avg_us_eager_pass": None if eager_us is None else round(eager_us, 2),
            "alg_bytes_per_launch": int(nbytes / n), "alg_flops_per_launch": int(flops / n),
            "hbm_frac": round(f_hbm, 4), "mfma_frac": round(f_mfma, 4),
            "mfma_peak_note": (
                "f32-equivalent peak of the instruction mix: every fp32 product as three fp16 "
                "MFMA products of two-part (hi/lo) fp16 splits, priced at the dense fp16 rate "
                "(16x the 157.3 TF f32 MFMA rate) / 3; both layers' products (k_fwd2: root + "
                "neighbour of layer 0 on the edge-row complement, both layer-1 products)"
                if name == "sage2_fwd" else
                "f32-equivalent peak of the instruction mix: root term 6 bf16 "
                "products per f32 product (16x the 157.3 TF f32 MFMA rate), "
                "neighbour term f32 MFMA; a layer on the 64-row fallback kernel "
                "(exact f32 MFMA throughout) is priced at the 157.3 TF f32 peak"),
            "all_kernels": {k: {"launches": v[0], "avg_us": round(1e3 * v[1] / v[0], 2),
                                "GBps": round(v[2] / (v[1] * 1e-3) / 1e9, 1),
                                "TFps": round(v[3] / (v[1] * 1e-3) / 1e12, 2),
                                "hbm_frac": round(v[2] / (HBM_PEAK_GBS * 1e9) / (v[1] * 1e-3), 4),
                                "mfma_frac": round(v[4] / (v[1] * 1e-3), 4)}
                            for k, v in summ.items()}})

    # the reference loop verbatim on the eager path (INTEGRATION Option B):
    # what a user gets without GraphedTrainStep / ngnn.optim.Adam
    eager_ref = None
    if rank == 0 and world == 1 and not args.no_eager_ref and ct is None:
        timed = [batches[(args.warmup + i) % nb] for i in range(args.steps)]
        ms_core = eager_reference_loop(timed, args, F_in, C, layers, dev, args.steps)
        ms_verb = eager_reference_loop(timed, args, F_in, C, layers, dev, args.steps, verbatim=True)
        ms_nadam = eager_reference_loop(timed, args, F_in, C, layers, dev, args.steps, ngnn_adam=True)
        graph_ms = 1e3 * dt / args.steps
        eager_ref = {
            "ms_per_step": round(ms_core, 4),
            "value": round(sum(layers * b.edge_index.shape[1] for b in timed) / args.steps / (ms_core * 1e-3), 1),
            "unit": "edges/s", "vs_graph_step": round(ms_core / graph_ms, 3),
            "ms_per_step_with_host_reads": round(ms_verb, 4),
            "ms_per_step_ngnn_adam": round(ms_nadam, 4),
            "vs_graph_step_ngnn_adam": round(ms_nadam / graph_ms, 3),
            "note": "pipeline.py:152-169 after the INTEGRATION.md Option-B swap: model(x, edge_index)"
                    "[:batch_size], F.cross_entropy, zero_grad, backward, torch.optim.Adam; no capture, "
                    "no loss head, no Adam fold (with_host_reads: + the loop's float(loss) and accuracy "
                    "count per step; ngnn_adam: the same loop with ngnn.optim.Adam constructed in place "
                    "of torch.optim.Adam, model.py:66-69).  Host-bound: torch.optim.Adam's foreach "
                    "step alone is ~0.1 ms of host time per step (torch.profiler, DESIGN.md 8d); "
                    "the two-layer stack runs as one C++ autograd node when ngnn_eager.so is "
                    "built (eager_cpp_node)",
            "eager_cpp_node": _eager_node_loaded()}

    # full epoch incl. GPU sampling (this rank's shard)
    epoch_s = epoch_sync = None
    if not args.no_epoch:
        # the synchronous loader: the host reads every block's counts (one
        # event wait per batch, one batch ahead)
        barrier()
        t1 = time.perf_counter()
        for b in loader:
            run(b)
        barrier()
        epoch_sync = epoch_s = time.perf_counter() - t1
        if graph and ct is None:
            gstep.check_inputs()  # (every batch of the epoch met the slot's contract)
            # the sync-free loader (ABI 19): blocks in capacity-sized buffers,
            # counts read by the slot load on the device -- no host wait at all
            loader_sf = NeighborLoader(graph_data, graph_data.train_idx, fanout, args.batch_size, shuffle=True,
                                       seed=7, rank=rank, world_size=world,
                                       gather_features=args.gather == "loader", sync_free=True)
            barrier()
            t1 = time.perf_counter()
            for b in loader_sf:
                run(b)
            barrier()
            epoch_s = time.perf_counter() - t1
            gstep.check_inputs()
    # the same epoch with the fused x[n_id] gather (batches carry the feature
    # table + n_id, the layer-0 kernels read the rows): no 61 MB row copy per
    # batch in the sampler, a few us more in the step -- reported beside
    epoch_fg = None
    if not args.no_epoch and graph and ct is None and args.gather == "loader" and world == 1:
        from ngnn.graphs import GraphedTrainStep, slot_size
        b0 = next(iter(NeighborLoader(graph_data, graph_data.train_idx, fanout, args.batch_size, shuffle=True,
                                      seed=7, rank=rank, world_size=world, gather_features=False)))
        loader_fg = NeighborLoader(graph_data, graph_data.train_idx, fanout, args.batch_size, shuffle=True,
                                   seed=7, rank=rank, world_size=world, gather_features=False, sync_free=True)
        n_cap, e_cap = slot_size(args.batch_size, fanout)
        gstep_fg = GraphedTrainStep(model, opt, args.batch_size, n_cap, e_cap, b0.x.size(1), dev, reducer=reducer)
        gstep_fg.capture(b0.x, b0.edge_index, b0.y)
        del b0
        if gstep_fg.x_rows:  # (the step took the indexed rows: the fused gather ran)
            barrier()
            t1 = time.perf_counter()
            for b in loader_fg:
                gstep_fg(b.x, b.edge_index, b.y, b.batch_size)
            barrier()
            epoch_fg = time.perf_counter() - t1
            gstep_fg.check_inputs()
        del gstep_fg

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and ct is None:
        cpu = cpu_baseline(batches, args, layers)

    if rank == 0:
        E_avg = sum(b.edge_index.shape[1] for b in batches) / nb
        N_avg = sum(b.num_nodes for b in batches) / nb
        line = {
            "metric": "aggregated edges/sec (GraphSAGE train step), ogbn-products fanout=[15,10] bs=1024"
                      if (args.dataset, args.fanout, args.batch_size) == ("ogbn-products", "15,10", 1024)
                      and ct is None
                      else f"aggregated edges/sec (co-teaching train step: 2 SAGE models + CTLoss), "
                           f"{args.dataset} fanout=[{args.fanout}] bs={args.batch_size}" if ct is not None
                      else f"aggregated edges/sec (GraphSAGE train step), {args.dataset} "
                           f"fanout=[{args.fanout}] bs={args.batch_size}",
            "value": round(edges / dt, 1), "unit": "edges/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * dt / args.steps, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": f"synthetic (seeded Chung-Lu graph with {args.dataset} sizes; random features)",
            "config": {"workload": workload,
                       "model": (f"SimpleGCN({F_in},{args.hidden},{C},L={layers}) sum-aggr + Adam(1e-3)"
                                 if args.module == "gcn" else
                                 f"2 x SAGE({F_in},{args.hidden},{C},L={layers}) {args.aggr}-aggr + CTLoss + "
                                 f"2 x Adam(1e-3)" if ct is not None else
                                 f"SAGE({F_in},{args.hidden},{C},L={layers}) {args.aggr}-aggr + Adam(1e-3)"),
                       "global_batch": args.batch_size * world, "fanout": fanout,
                       "avg_edges_per_batch": round(E_avg), "avg_nodes_per_batch": round(N_avg),
                       "parallelism": f"dp{world} (seed-sharded, {_allreduce_name(world)} grad all-reduce)"},
            "host_issue_ms_per_step": round(1e3 * t_issue / args.steps, 4),
            "launch": "eager" if not graph else "hip-graph replay (step captured once)",
            "feature_gather": ("fused x[n_id] in the layer-0 kernels" if args.gather == "fused"
                               and graph and gstep.x_rows else "loader copies x[n_id]"),
            # the epoch as the framework runs it best: the sync-free loader with
            # the fused x[n_id] gather when it ran (graph mode), the other
            # epoch configurations beside it
            "epoch_time_s": round(epoch_fg, 4) if epoch_fg is not None else (
                None if epoch_s is None else round(epoch_s, 4)),
            "epoch_mode": ("sync-free loader, fused x[n_id] gather" if epoch_fg is not None else
                           "sync-free loader, loader row copy" if (graph and ct is None and epoch_s is not None)
                           else "loader (host reads each block's counts)"),
            "epoch_time_s_sync_free_row_copy": None if (epoch_s is None or epoch_s is epoch_sync) else round(epoch_s, 4),
            "epoch_time_s_sync_loader": None if epoch_sync is None else round(epoch_sync, 4),
            "epoch_batches_per_rank": len(loader),
            "allreduce": ar,
            "eager_drop_in": eager_ref,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
