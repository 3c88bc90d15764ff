"""Per-launch timing of ngnn_sage2_fwd on the headline block (ogbn-products
sizes, fanout [15, 10], batch 1024, train-mode dropout 0.5): each stage run
alone REPS times between HIP events on the library's stream.

    python tools/fwd2_micro.py [--reps 50] [--stages edge,main,narrow]

With NGNN_LIB=dbg/libngnn_dbg.so (tools/build_dbg.sh) and NGNN_FWD2_DBG=k
it times k_fwd2's attribution variants (bits: 1 no reduce, 2 no layer-1
products, 4 no layer-0 products, 8 no x split).  Profiling aid only.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "noise-gnn_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

import ngnn  # noqa: E402
from ngnn import _lib, fused  # noqa: E402
from ngnn.block import get_block  # noqa: E402
from ngnn.loader import sample_block, synthetic_graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--stages", default="edge,main,narrow")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--dbg", default="", help="comma list of NGNN_FWD2_DBG values to time 'main' under")
    ap.add_argument("--edge-dbg", default="", help="comma list of NGNN_EDGE_DBG values to time 'edge' under")
    ap.add_argument("--head", action="store_true", help="the narrow stage with the loss head (fused.LossHead)")
    ap.add_argument("--head-dbg", default="", help="comma list of NGNN_HEAD_DBG values to time 'narrow' under")
    ap.add_argument("--all-h", action="store_true",
                    help="write h for every row (default: rows < n_edge_rows, the step's R' bound)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    graph = synthetic_graph("ogbn-products", dev, seed=0, scale=args.scale)
    torch.manual_seed(0)
    seeds = graph.train_idx[torch.randperm(graph.train_idx.numel(), device=dev)[:1024]]
    b = sample_block(graph, seeds, [15, 10], seed=1)
    blk = get_block(b.edge_index, b.num_nodes)
    model = ngnn.SAGE(b.x.size(1), 256, 47, 2, dropout=0.5).to(dev)
    c0, c1 = model.convs
    params = [c0.lin_l.weight, c0.lin_l.bias, c0.lin_r.weight, c1.lin_l.weight, c1.lin_l.bias, c1.lin_r.weight]
    assert fused.sage2_ok(b.x, blk, "mean", params, False), "not the sage2 shape"
    if not args.all_h:  # h rows as in the step: the slot's R' (rows with in-edges)
        n_e_ = int(blk.n_active or 0)
        blk.r_next = (torch.tensor([n_e_], dtype=torch.int32, device=dev), n_e_, True)
    seed = 12345
    head = None
    if args.head:
        y = torch.randint(0, 47, (1024,), device=dev)
        n_e0 = int(blk.n_active or 0)
        lh = fused.LossHead(y, 1024, b.num_nodes, 47, torch.tensor([n_e0], dtype=torch.int32, device=dev))
        head = lh.start()
    bufs = fused.sage2_forward(b.x, blk, "mean", params, 0.5, seed, None, head=head)[:3]
    torch.cuda.synchronize()
    st = {"edge": _lib.SAGE2_EDGE, "main": _lib.SAGE2_MAIN, "narrow": _lib.SAGE2_NARROW,
          "fused": _lib.SAGE2_EDGE | _lib.SAGE2_MAIN}  # (fused: k_fwd2x, as the step runs it)
    n_e = int(blk.n_active or 0)
    print(f"block: N={b.num_nodes} E={b.edge_index.size(1)} n_edge_rows={n_e} "
          f"dbg={os.environ.get('NGNN_FWD2_DBG', '-')}")
    runs = [(n, None, None) for n in args.stages.split(",")]
    runs += [("main", "NGNN_FWD2_DBG", v) for v in args.dbg.split(",") if v]
    runs += [("edge", "NGNN_EDGE_DBG", v) for v in args.edge_dbg.split(",") if v]
    runs += [("narrow", "NGNN_HEAD_DBG", v) for v in args.head_dbg.split(",") if v]
    for name, env, dbg in runs:
        os.environ.pop("NGNN_FWD2_DBG", None)
        os.environ.pop("NGNN_EDGE_DBG", None)
        os.environ.pop("NGNN_HEAD_DBG", None)
        if dbg is not None:
            os.environ[env] = dbg
        for _ in range(5):
            fused.sage2_forward(b.x, blk, "mean", params, 0.5, seed, None, stages=st[name], bufs=bufs,
                                    head=head if name == "narrow" else None)
        torch.cuda.synchronize()
        # the REPS launches as one graph (no host issue between them)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(args.reps):
                fused.sage2_forward(b.x, blk, "mean", params, 0.5, seed, None, stages=st[name], bufs=bufs,
                                    head=head if name == "narrow" else None)
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        tag = name if dbg is None else f"{name}/dbg{dbg}"
        print(f"{tag:12s} {e0.elapsed_time(e1) * 1e3 / args.reps:8.1f} us/launch (graph of back-to-back launches)", flush=True)


if __name__ == "__main__":
    main()
