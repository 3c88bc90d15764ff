"""Host time per section of the eager reference loop (pipeline.py:152-169
after the Option-B swap): forward / loss / zero_grad / backward / optimizer
step of the loop, and inside them ngnn's own Python (block lookup, the stack
node's forward and backward, the two-layer launches' wrappers) -- wall time
on the host with the device running behind (the loop is host-bound).

    python tools/eager_sections.py [--steps 200] [--ngnn-adam]"""
import argparse
import collections
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "noise-gnn_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import ngnn  # noqa: E402
from ngnn import block as nblock  # noqa: E402
from ngnn import fused, models  # noqa: E402
from ngnn.loader import NeighborLoader, synthetic_graph  # noqa: E402

acc = collections.defaultdict(float)
cnt = collections.defaultdict(int)


def timed(name, fn):
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            acc[name] += time.perf_counter() - t0
            cnt[name] += 1
    return w


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--ngnn-adam", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = synthetic_graph("ogbn-products", dev, seed=0)
    loader = NeighborLoader(g, g.train_idx, [15, 10], 1024, shuffle=True, seed=7)
    it = iter(loader)
    batches = [next(it) for _ in range(6)]
    torch.manual_seed(1234)
    model = ngnn.SAGE(100, 256, 47, 2, dropout=0.5).to(dev).train()
    from ngnn.optim import Adam as NgnnAdam
    opt = (NgnnAdam if a.ngnn_adam else torch.optim.Adam)(model.parameters(), lr=1e-3)
    # ngnn's own Python inside the loop
    models.get_block = timed("get_block", nblock.get_block)
    fused.sage2_forward = timed("sage2_forward", fused.sage2_forward)
    fused.sage2_backward = timed("sage2_backward", fused.sage2_backward)
    fused._SAGEStack.backward = staticmethod(timed("stack.backward", fused._SAGEStack.backward))
    fused._SAGEStack.forward = staticmethod(timed("stack.forward", fused._SAGEStack.forward))
    models._dropout_seed = timed("dropout_seed", models._dropout_seed)
    fused.sage_stack = timed("sage_stack", fused.sage_stack)
    fused._eager_sage2 = timed("eager_sage2 (C++ node)", fused._eager_sage2)

    def one(b, rec):
        t = [time.perf_counter()]
        out = model(b.x, b.edge_index)[:b.batch_size]
        t.append(time.perf_counter())
        loss = F.cross_entropy(out, b.y[:b.batch_size])
        t.append(time.perf_counter())
        opt.zero_grad()
        t.append(time.perf_counter())
        loss.backward()
        t.append(time.perf_counter())
        opt.step()
        t.append(time.perf_counter())
        if rec:
            for n, x0, x1 in zip(("forward", "loss", "zero_grad", "backward", "opt.step"), t, t[1:]):
                acc["loop." + n] += x1 - x0
                cnt["loop." + n] += 1

    for i in range(10):
        one(batches[i % len(batches)], False)
    torch.cuda.synchronize()
    acc.clear()
    cnt.clear()
    t0 = time.perf_counter()
    for i in range(a.steps):
        one(batches[i % len(batches)], True)
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    tw = time.perf_counter() - t0
    print(f"eager step {1e3 * tw / a.steps:.3f} ms wall, host issue {1e3 * th / a.steps:.3f} ms "
          f"({'ngnn' if a.ngnn_adam else 'torch'} Adam)")
    for k in sorted(acc, key=lambda k: -acc[k]):
        print(f"  {k:22s} {1e6 * acc[k] / a.steps:8.1f} us/step  ({cnt[k] / a.steps:.1f} calls)")


if __name__ == "__main__":
    main()
