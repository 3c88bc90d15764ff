"""Diagnostic: per-segment cycle sums of k_root from a NGNN_ROOT_TRACE=1 build
(NGNN_LIB=ablib/<variant>.so): one L0 launch shape (products, edge-free block).

    NGNN_LIB=ablib/trace.so python tools/root_trace.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "noise-gnn_amd"))
import torch  # noqa: E402


def main():
    from ngnn import _lib
    from ngnn.block import Block
    from ngnn.fused import sage_layer_fwd
    from ngnn.loader import sample_block, synthetic_graph
    lib = _lib.load()
    fn = lib.ngnn_debug_root_trace
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    dev = torch.device("cuda:0")
    g = synthetic_graph("ogbn-products", dev, seed=0)
    b = sample_block(g, g.train_idx[:1024], [15, 10], seed=1)
    N = b.num_nodes
    empty = Block(torch.empty(2, 0, dtype=torch.long, device=dev), N)
    empty.n_active = 0
    out = {}
    for name, x, K, Fo, relu, p in (("L0", b.x, 100, 256, True, 0.5), ("L0_nodrop", b.x, 100, 256, True, 0.0)):
        wl = torch.randn(Fo, K, device=dev) * 0.1
        wr = torch.randn(Fo, K, device=dev) * 0.1
        bl = torch.randn(Fo, device=dev)
        for _ in range(3):
            sage_layer_fwd(x, empty, "mean", wl, bl, wr, relu=relu, p_drop=p, seed=7)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 8)()
        fn(buf)
        reps = 10
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            sage_layer_fwd(x, empty, "mean", wl, bl, wr, relu=relu, p_drop=p, seed=7)
        e1.record()
        torch.cuda.synchronize()
        fn(buf)
        out[name + "_us"] = round(e0.elapsed_time(e1) * 1e3 / reps, 2)
        tiles = max(buf[3], 1)
        out[name] = {"tiles": buf[3] // reps, "cyc_per_tile": {"head_tail": buf[0] / tiles,
                     "root": buf[1] / tiles, "epilogue": buf[2] / tiles}, "prologue_per_wave": buf[4] / 1024}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
