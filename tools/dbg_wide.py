"""Debug: (K, Fo) layer variants (agg_out / n_rows_dev / dropout) vs the oracle."""
import sys
sys.path.insert(0, "noise-gnn_amd"); sys.path.insert(0, "."); sys.path.insert(0, "tests")
import torch
from ngnn.block import Block
from ngnn.fused import sage_layer_fwd, agg_buffer
from oracle import pyg_ref
from test_gpu_fused import rand_block, dropout_keep, dropout_scale
DEV = "cuda"
K, Fo = int(sys.argv[1]), int(sys.argv[2])
red = sys.argv[3] if len(sys.argv) > 3 else "max"
N = 1100
g = torch.Generator().manual_seed(K + Fo)
ei = rand_block(K * 5 + Fo, N, 6000)
ei = ei[:, ei[1] < 700]
x = torch.randn(N, K, generator=g)
conv = pyg_ref.SAGEConv(K, Fo, aggr=red)
with torch.no_grad():
    pre = conv(x, ei).relu()
for p in (0.0, 0.5):
    want = pre * dropout_keep(77, N, Fo, p) * dropout_scale(p) if p else pre
    for use_agg in (True, False):
        for use_nrd in (False, True):
            blk = Block(ei.to(DEV), N)
            blk.n_active = 700
            if use_nrd:
                blk.n_rows_dev = torch.tensor([900], dtype=torch.int32, device=DEV)
            agg = agg_buffer(N, K, DEV, Fo) if use_agg else None
            got = sage_layer_fwd(x.to(DEV), blk, red, conv.lin_l.weight.to(DEV), conv.lin_l.bias.to(DEV),
                                 conv.lin_r.weight.to(DEV), relu=True, p_drop=p, seed=77, agg_out=agg).cpu()
            n = 900 if use_nrd else N
            d = (got[:n] - want[:n]).abs()
            bad = d > 1e-4
            rows = bad.any(1).nonzero().flatten()
            cols = bad.any(0).nonzero().flatten()
            print(f"p={p} agg={use_agg} nrd={use_nrd}: max err {d.max():.3g}, bad rows {len(rows)} "
                  f"[{rows[:5].tolist()}..{rows[-3:].tolist() if len(rows) else ''}] bad cols {cols.tolist()[:40]}")
