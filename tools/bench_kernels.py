"""Micro-benchmark of the fused SAGE kernels on one products-[15,10] block.

Times (HIP events, median of --reps) the forward layer kernel in several
modes to separate gather, GEMM, epilogue and dropout costs, plus the
backward pieces.  Run on the GPU box:

    python tools/bench_kernels.py [--reps 20] [--scale 1.0]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "noise-gnn_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def timeit(fn, reps):
    """Average GPU time per call over `reps` back-to-back calls between two
    events (the kernels are far longer than the host enqueue, so the queue
    stays full and host overhead is not measured)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = None
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) * 1e3 / reps
        best = t if best is None else min(best, t)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--scale", type=float, default=1.0)
    a = ap.parse_args()
    from ngnn.block import Block
    from ngnn.fused import _gemm_layer, pack_weight
    from ngnn.loader import sample_block, synthetic_graph
    dev = torch.device("cuda:0")
    g = synthetic_graph("ogbn-products", dev, seed=0, scale=a.scale)
    b = sample_block(g, g.train_idx[:1024], [15, 10], seed=1)
    N, E = b.num_nodes, b.edge_index.shape[1]
    blk = Block(b.edge_index, N)
    empty = Block(torch.empty(2, 0, dtype=torch.long, device=dev), N)
    res = {"N": N, "E": E, "n_active": b.n_id.numel()}
    torch.manual_seed(0)
    for (K, Fo) in [(100, 256), (256, 47)]:
        x = torch.randn(N, K, device=dev)
        wl = torch.randn(Fo, K, device=dev) * 0.1
        wr = torch.randn(Fo, K, device=dev) * 0.1
        bl = torch.randn(Fo, device=dev)
        agg = torch.empty(N, K, device=dev)
        out = torch.empty(N, Fo, device=dev)
        pl, pr = pack_weight(wl), pack_weight(wr)
        tag = f"K{K}_F{Fo}"

        def layer(block, relu, p, agg_out):
            return lambda: _gemm_layer(x, K, N, block, "mean", pl, pr, bl, Fo, out, relu, p, 7,
                                       agg_out=agg_out)
        res[tag + "_full_drop"] = timeit(layer(blk, True, 0.5, agg), a.reps)
        res[tag + "_full"] = timeit(layer(blk, True, 0.0, agg), a.reps)
        res[tag + "_noagg_out"] = timeit(layer(blk, True, 0.0, None), a.reps)
        res[tag + "_root_only"] = timeit(layer(empty, False, 0.0, None), a.reps)
        res[tag + "_root_only_drop"] = timeit(layer(empty, True, 0.5, None), a.reps)
        # raw-weight entry (the model's path): split at n_active (dense kernel
        # for the edge-free rows) vs no split, and the dense kernel alone
        from ngnn.fused import sage_layer_fwd
        n_act = int(b.edge_index[1].max().item()) + 1
        blk_s = Block(b.edge_index, N)
        blk_s.n_active = n_act

        def raw(block, p):
            return lambda: sage_layer_fwd(x, block, "mean", wl, bl, wr, relu=True, p_drop=p,
                                          seed=7, agg_out=agg)
        res[tag + "_raw_drop_nosplit"] = timeit(raw(blk, 0.5), a.reps)
        res[tag + "_raw_drop_split"] = timeit(raw(blk_s, 0.5), a.reps)
        blk_e = Block(torch.empty(2, 0, dtype=torch.long, device=dev), N)
        blk_e.n_active = 0
        res[tag + "_dense_only_drop"] = timeit(raw(blk_e, 0.5), a.reps)
        res[tag + "_dense_only"] = timeit(raw(blk_e, 0.0), a.reps)
        res["n_active"] = n_act
        res[tag + "_pack2"] = timeit(lambda: (pack_weight(wl), pack_weight(wr)), a.reps)
        # pure-copy roofline reference: read x + write out
        res[tag + "_torch_copy_x"] = timeit(lambda: x.clone(), a.reps)
        res[tag + "_torch_mm_root"] = timeit(lambda: torch.mm(x, wr.t(), out=out), a.reps)
        res[tag + "_gflop_root"] = 2 * N * K * Fo / 1e9
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
