import sys, torch
sys.path.insert(0, "noise-gnn_amd")
from ngnn import _lib
lib = _lib.load()
dev = torch.device("cuda:0")
n = 1_490_000 * 47
x = torch.randn(n, device=dev)
y = torch.empty(n, dtype=torch.bfloat16, device=dev)
def ours():
    lib.ngnn_cast_f32_bf16(_lib.ptr(x), _lib.ptr(y), n, _lib.stream_handle(dev))
def aten():
    y.copy_(x)
for name, f in (("ngnn", ours), ("aten", aten), ("ngnn", ours)):
    for _ in range(3): f()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20): f()
    g.replay(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); g.replay(); e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    print(f"{name}: {us:.1f} us  {6*n/us/1e6:.2f} TB/s", flush=True)
