"""Timing aid for ngnn.optim.Adam's launch on Amazon-Computers' parameter set
(SAGE(767, 512, 10): ~0.8 M parameters in six tensors): the step captured in
a HIP graph, 50 replays between HIP events.  Profiling aid only."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "noise-gnn_amd"))
import torch  # noqa: E402

from ngnn.optim import Adam  # noqa: E402


def main(reps=50, scale=1.0):
    dev = torch.device("cuda:0")
    shapes = [(max(1, int(512 * scale)), 767), (512,), (max(1, int(512 * scale)), 767), (10, 512), (10,), (10, 512)]
    ps = [torch.randn(s, device=dev, requires_grad=True) for s in shapes]
    for p in ps:
        p.grad = torch.randn_like(p)
    opt = Adam(ps, lr=1e-3)
    opt.step()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        opt.step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(reps):
            opt.step()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    n = sum(p.numel() for p in ps)
    print(f"adam step {e0.elapsed_time(e1) * 1e3 / reps:8.2f} us/launch (graph of {reps}, {n} parameters)")


if __name__ == "__main__":
    main(scale=float(sys.argv[1]) if len(sys.argv) > 1 else 1.0)
