"""Host-side cost of one bench training step (cProfile over K steps, no
syncs inside), to see where the Python/launch time goes.
    python tools/host_profile.py [--steps 50]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "noise-gnn_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--timer", action="store_true", help="keep the per-launch event timer on")
    a = ap.parse_args()
    import bench
    import ngnn
    from ngnn import _timing
    from ngnn.distributed import GradAllReduce
    from ngnn.loader import NeighborLoader, synthetic_graph
    dev = torch.device("cuda:0")
    g = synthetic_graph("ogbn-products", dev, seed=0)
    torch.manual_seed(1234)
    model = ngnn.SAGE(100, 256, 47, 2, dropout=0.5).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)
    red = GradAllReduce(model.parameters())
    loader = NeighborLoader(g, g.train_idx, [15, 10], 1024, shuffle=True, seed=7)
    it = iter(loader)
    batches = [next(it) for _ in range(8)]
    for i in range(10):
        bench.train_step(model, opt, red, batches[i % 8])
    torch.cuda.synchronize()
    timer = _timing.KernelTimer() if a.timer else None
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    if timer:
        timer.__enter__()
    pr.enable()
    for i in range(a.steps):
        bench.train_step(model, opt, red, batches[i % 8])
    pr.disable()
    t1 = time.perf_counter()
    if timer:
        timer.__exit__(None, None, None)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host issue {1e3 * (t1 - t0) / a.steps:.3f} ms/step, wall {1e3 * (t2 - t0) / a.steps:.3f} ms/step")
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)


if __name__ == "__main__":
    main()
