"""The whole-block sampler alone (ngnn_sample_block + _finish) on the
products-shaped graph, one block at a time (synchronised between blocks), for
rocprofv3 --kernel-trace: per-launch durations by position in the block's
launch sequence (tools/sampler_micro.py --trace CSV prints them).

    python tools/sampler_micro.py [--blocks 30] [--fanout 15,10] [--bs 1024]
    python tools/sampler_micro.py --trace run_kernel_trace.csv"""
import argparse
import collections
import csv
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "noise-gnn_amd"))


def trace(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    blocks, cur = [], None
    for r in rows:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        name = name.replace("ngnn::", "")
        if "k_sb_init" in name:
            cur = []
            blocks.append(cur)
        if cur is not None and "k_sb" in name:
            cur.append((name, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
                        int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    blocks = blocks[3:]  # (warm-up)
    by = collections.defaultdict(list)
    spans = []
    for b in blocks:
        for i, (n, d, _, _) in enumerate(b):
            by[(i, n)].append(d)
        spans.append((b[-1][3] - b[0][2]) / 1e3)
    print(f"blocks analysed: {len(blocks)}; first-to-last launch span median {statistics.median(spans):.1f} us")
    tot = 0.0
    for (i, n), v in sorted(by.items()):
        m = statistics.median(v)
        tot += m
        print(f"  {i:2d} {n:40s} {m:8.1f} us")
    print(f"  sum of medians {tot:.1f} us")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=30)
    ap.add_argument("--fanout", default="15,10")
    ap.add_argument("--bs", type=int, default=1024)
    ap.add_argument("--trace")
    a = ap.parse_args()
    if a.trace:
        return trace(a.trace)
    import torch
    from ngnn.loader import sample_block, synthetic_graph
    dev = torch.device("cuda:0")
    g = synthetic_graph("ogbn-products", dev, seed=0)
    fan = [int(f) for f in a.fanout.split(",")]
    perm = g.train_idx[torch.randperm(g.train_idx.numel(), device=dev)]
    ts = []
    for b in range(a.blocks):
        s = perm[(b * a.bs) % (perm.numel() - a.bs):][:a.bs]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        blk = sample_block(g, s, fan, seed=b)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    print(f"sample_block wall median {1e6 * statistics.median(ts[3:]):.1f} us "
          f"(nodes {blk.num_nodes}, edges {blk.edge_index.size(1)})")


if __name__ == "__main__":
    main()
