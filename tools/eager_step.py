"""The reference loop (pipeline.py:152-169) on ngnn's modules, eager, no
capture: the bench's eager_drop_in field as a standalone run for rocprofv3
(kernel list) and torch.profiler (host time per op).
    python tools/eager_step.py [--steps 30] [--host-prof]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "noise-gnn_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import ngnn  # noqa: E402
from ngnn.loader import NeighborLoader, synthetic_graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--host-prof", action="store_true")
    ap.add_argument("--cprofile", action="store_true")
    ap.add_argument("--ngnn-adam", action="store_true", help="ngnn.optim.Adam in place of torch.optim.Adam")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = synthetic_graph("ogbn-products", dev, seed=0)
    loader = NeighborLoader(g, g.train_idx, [15, 10], 1024, shuffle=True, seed=7)
    it = iter(loader)
    batches = [next(it) for _ in range(10)]
    torch.manual_seed(1234)
    model = ngnn.SAGE(100, 256, 47, 2, dropout=0.5).to(dev).train()
    from ngnn.optim import Adam as NgnnAdam
    opt = (NgnnAdam if a.ngnn_adam else torch.optim.Adam)(model.parameters(), lr=1e-3)

    def one(b):
        out = model(b.x, b.edge_index)[:b.batch_size]
        loss = F.cross_entropy(out, b.y[:b.batch_size])
        opt.zero_grad()
        loss.backward()
        opt.step()

    for i in range(5):
        one(batches[i % 10])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        one(batches[i % 10])
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"eager step {1e3 * dt / a.steps:.3f} ms (host issue {1e3 * t_issue / a.steps:.3f} ms)")
    if a.cprofile:
        import cProfile
        import pstats
        # (backward on the calling thread, so the profile sees its Python)
        torch.autograd.set_multithreading_enabled(False)
        pr = cProfile.Profile()
        pr.enable()
        for i in range(50):
            one(batches[i % 10])
        torch.cuda.synchronize()
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(35)
    if a.host_prof:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU]) as p:
            for i in range(10):
                one(batches[i % 10])
            torch.cuda.synchronize()
        print(p.key_averages().table(sort_by="cpu_time_total", row_limit=40))


if __name__ == "__main__":
    main()
