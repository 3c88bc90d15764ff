"""Timing aid for ngnn_sage2_bwd on headline-sized bounds (R = 1024 seeds,
R' = 16 k rows of N = 150 k; K0 = 100, F1 = 47): REPS back-to-back calls
between HIP events.  Synthetic inputs as tests/test_gpu_bwd2.py builds them
(device-side, no host reference).  Profiling aid only."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "noise-gnn_amd"))
import torch  # noqa: E402

from ngnn import _lib  # noqa: E402


def main(reps=50):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    N, R, Rn, K0, F1 = 150_000, 1024, 16_000, 100, 47
    deg = torch.randint(0, 16, (Rn,), generator=g, device=dev)
    rowptr = torch.zeros(N + 1, dtype=torch.int32, device=dev)
    rowptr[1:Rn + 1] = torch.cumsum(deg, 0).to(torch.int32)
    rowptr[Rn + 1:] = rowptr[Rn]
    E = int(rowptr[-1])
    dst = torch.repeat_interleave(torch.arange(Rn, device=dev), deg)
    src = torch.where(dst < R, torch.randint(0, Rn, (E,), generator=g, device=dev),
                      torch.randint(0, N, (E,), generator=g, device=dev))
    col = src.to(torch.int32)
    dy = torch.zeros(N, F1, device=dev)
    dy[:R] = torch.randn(R, F1, generator=g, device=dev) * 1e-3
    h = torch.relu(torch.randn(N, 256, generator=g, device=dev))
    x = torch.randn(N, K0, generator=g, device=dev)
    agg0 = torch.randn(N, K0, generator=g, device=dev)
    wl1 = torch.randn(F1, 256, generator=g, device=dev) * 0.05
    wr1 = torch.randn(F1, 256, generator=g, device=dev) * 0.05
    out = [torch.empty(F1, 256, device=dev), torch.empty(F1, device=dev), torch.empty(F1, 256, device=dev),
           torch.empty(256, K0, device=dev), torch.empty(256, device=dev), torch.empty(256, K0, device=dev)]
    bounds = torch.tensor([R, Rn], dtype=torch.int32, device=dev)
    lib = _lib.load()
    ws = torch.zeros(lib.ngnn_sage2_bwd_workspace_bytes(N, K0, F1), dtype=torch.uint8, device=dev)

    def call():
        rc = lib.ngnn_sage2_bwd(_lib.ptr(dy), F1, F1, _lib.ptr(wl1), _lib.ptr(wr1), 256, _lib.ptr(h), 256, 2.0,
                                _lib.ptr(x), None, None, None, 0, K0, K0, _lib.ptr(agg0), K0,
                                _lib.ptr(rowptr), _lib.ptr(col), N, bounds.data_ptr(), bounds.data_ptr() + 4,
                                _lib.REDUCE["mean"], *(_lib.ptr(o) for o in out), None, None, _lib.ptr(ws), ws.numel(),
                                _lib.stream_handle(dev))
        assert rc == _lib.OK, rc
    for _ in range(5):
        call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        call()
    e1.record()
    torch.cuda.synchronize()
    print(f"ngnn_sage2_bwd {e0.elapsed_time(e1) * 1e3 / reps:8.1f} us/call (3 launches, incl. host issue)")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50)
