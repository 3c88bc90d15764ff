"""Debug: per-layer output gradients of the fused max stack vs the oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "noise-gnn_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import ngnn  # noqa: E402
from ngnn import fused  # noqa: E402
from oracle import pyg_ref  # noqa: E402

dev = torch.device("cuda:0")
from ngnn.loader import sample_block, synthetic_graph  # noqa: E402
for H in (192, 256):
    g = synthetic_graph("ogbn-arxiv", dev, seed=0)
    b = sample_block(g, g.train_idx[:1024], [15, 10], seed=5)
    torch.manual_seed(2)
    mine = ngnn.SAGE(128, H, 40, 2, aggr="max").to(dev).eval()
    ref = pyg_ref.SAGE(128, H, 40, 2, aggr="max").eval()
    ref.load_state_dict({k: v.cpu() for k, v in mine.state_dict().items()})
    fused._debug_grads = []
    out = mine(b.x, b.edge_index)
    F.cross_entropy(out[:1024], b.y[:1024]).backward()
    dbg = fused._debug_grads
    fused._debug_grads = None
    # oracle with the intermediate kept
    x = b.x.cpu()
    ei = b.edge_index.cpu()
    h0 = ref.convs[0](x, ei)
    h1 = h0.relu()
    h1.retain_grad()
    o = ref.convs[1](h1, ei)
    F.cross_entropy(o[:1024], b.y[:1024].cpu()).backward()
    agg1_ref = pyg_ref.scatter(h1.detach()[ei[0]], ei[1], 0, h1.size(0), "max")
    for (i, dy, agg) in dbg:
        print("H", H, "layer", i, "dy shape", tuple(dy.shape))
    dh1 = dbg[1][1].cpu()  # layer 0's output gradient (before the mask)
    has = torch.bincount(ei[1], minlength=h1.size(0)) > 0
    agg1 = dbg[0][2].cpu()
    print(" agg1 diff on edge rows", (agg1[has] - agg1_ref[has]).abs().max().item())
    d = (dh1 - h1.grad).abs()
    print(" dh1 max diff", d.max().item(), "at", divmod(int(d.argmax()), H), "ref max", h1.grad.abs().max().item())
    rows = (d > 1e-6).any(1).nonzero().view(-1)
    print(" rows with diff", rows.numel(), rows[:20].tolist())
    cols = (d > 1e-6).any(0).nonzero().view(-1)
    print(" cols with diff", cols.numel(), cols[:40].tolist())
