"""Probe: eager train step vs the same step captured in a HIP graph
(torch.cuda.CUDAGraph) on one static products-[15,10] block.
    python tools/graph_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "noise-gnn_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    import ngnn
    from ngnn.block import hint_edge_index
    from ngnn.loader import NeighborLoader, synthetic_graph
    dev = torch.device("cuda:0")
    g = synthetic_graph("ogbn-products", dev, seed=0)
    torch.manual_seed(1234)
    model = ngnn.SAGE(100, 256, 47, 2, dropout=0.5).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, fused=True, capturable=True)
    b = next(iter(NeighborLoader(g, g.train_idx, [15, 10], 1024, shuffle=True, seed=7)))
    x_s, ei_s, y_s = b.x.clone(), b.edge_index.clone(), b.y[:1024].clone()
    hint_edge_index(ei_s, dst_sorted=True, src_sorted=False)
    B = 1024

    def step():
        out = model(x_s, ei_s)[:B]
        loss = F.cross_entropy(out, y_s)
        opt.zero_grad(set_to_none=False)
        loss.backward()
        opt.step()
        return loss

    def timeit(fn, n=50):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        return 1e3 * (t1 - t0) / n, 1e3 * (t2 - t0) / n

    for _ in range(5):
        step()
    print("eager   issue/wall ms per step: %.3f %.3f" % timeit(step))
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    ngnn.block.block_cache.clear()
    hint_edge_index(ei_s, dst_sorted=True, src_sorted=False)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        loss = step()
    torch.cuda.synchronize()
    print("graph   issue/wall ms per step: %.3f %.3f" % timeit(gr.replay))
    print("loss after replays", float(loss))
    # timing events inside a capture (external=True -> event record nodes)
    try:
        from ngnn import _timing
        _timing.EXTERNAL = True
        gr2 = torch.cuda.CUDAGraph()
        timer = _timing.KernelTimer(only=["sage_fwd"])
        with timer:
            with torch.cuda.graph(gr2):
                step()
        print("timed graph issue/wall ms per step: %.3f %.3f" % timeit(gr2.replay))
        gr2.replay()
        torch.cuda.synchronize()
        print("timed capture OK", [(r.name, r.start.elapsed_time(r.end)) for r in timer.recs])
    except Exception as e:  # noqa: BLE001
        print("timed capture failed:", repr(e)[:400])


if __name__ == "__main__":
    main()
