"""Forward layer kernel timing on one full ogbn-products [15,10] bs 1024
block: the metric model's two layer shapes (L0 100->256 relu+dropout, L1
256->47) through ngnn_sage_fwd_raw, in the modes that separate its costs.
HIP events around `reps` back-to-back launches (median of 3 rounds).

    python tools/kbench_fwd.py [--reps 20] [--only L0_train_x3,...]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "noise-gnn_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / reps)
    return sorted(ts)[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    from ngnn.block import Block
    from ngnn.fused import exact_f32, sage_layer_fwd
    from ngnn.loader import sample_block, synthetic_graph
    dev = torch.device("cuda:0")
    g = synthetic_graph("ogbn-products", dev, seed=0)
    b = sample_block(g, g.train_idx[:1024], [15, 10], seed=1)
    N, E = b.num_nodes, b.edge_index.shape[1]
    blk = Block(b.edge_index, N)
    blk.n_active = int(b.edge_index[1].max()) + 1  # the sampler's row hint
    res = {"N": N, "E": E, "n_edge_rows": blk.n_active}
    torch.manual_seed(0)
    only = set(a.only.split(",")) if a.only else None
    h = torch.randn(N, 256, device=dev).relu()
    for tag, x, K, Fo, relu, p in (("L0", b.x, 100, 256, True, 0.5), ("L1", h, 256, 47, False, 0.0)):
        wl = torch.randn(Fo, K, device=dev) * 0.1
        wr = torch.randn(Fo, K, device=dev) * 0.1
        bl = torch.randn(Fo, device=dev)
        agg = torch.empty(N, K, device=dev)

        def run(p_=p, ex=False, blk_=blk, agg_=agg):
            def f():
                with exact_f32(ex):
                    sage_layer_fwd(x, blk_, "mean", wl, bl, wr, relu=relu, p_drop=p_, seed=7,
                                   agg_out=agg_)
            return f
        empty = Block(torch.empty(2, 0, dtype=torch.long, device=dev), N)
        empty.n_active = 0  # no row has in-edges (the kernel's root-term-only loop)
        def run_narrow():
            def f():
                sage_layer_fwd(x, blk, "mean", wl, bl, wr, relu=False, p_drop=0.0, seed=7,
                               narrow=True)
            return f
        cases = {f"{tag}_model_x3": run(), f"{tag}_model_exact": run(ex=True),
                 f"{tag}_narrow_x3": run_narrow(),
                 f"{tag}_nodrop_x3": run(p_=0.0), f"{tag}_noedges_x3": run(blk_=empty, agg_=None),
                 f"{tag}_noedges_nodrop_x3": run(p_=0.0, blk_=empty, agg_=None),
                 f"{tag}_noedges_exact": run(ex=True, blk_=empty, agg_=None)}
        for k, fn in cases.items():
            if only and k not in only:
                continue
            res[k] = round(timeit(fn, a.reps), 2)
        res[f"{tag}_torch_copy_x"] = round(timeit(lambda: x.clone(), a.reps), 2)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
