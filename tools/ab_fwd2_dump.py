"""Dump ngnn_sage2_fwd outputs (h, out, agg) on sampled products blocks, for
A/B comparison of two builds (NGNN_LIB).  python tools/ab_fwd2_dump.py OUT.pt"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "noise-gnn_amd"))
import torch  # noqa: E402

import ngnn  # noqa: E402
from ngnn import fused  # noqa: E402
from ngnn.block import get_block  # noqa: E402
from ngnn.loader import sample_block, synthetic_graph  # noqa: E402

dev = torch.device("cuda:0")
res = {}
for scale, bs in ((0.01, 256), (1.0, 1024)):
    graph = synthetic_graph("ogbn-products", dev, seed=2, scale=scale)
    b = sample_block(graph, graph.train_idx[:bs], [15, 10], seed=4)
    blk = get_block(b.edge_index, b.num_nodes)
    torch.manual_seed(11)
    m = ngnn.SAGE(100, 256, 47, 2, dropout=0.5).to(dev)
    params = [q.detach() for c in m.convs for q in (c.lin_l.weight, c.lin_l.bias, c.lin_r.weight)]
    for p in (0.0, 0.5, 0.25):
        h, out, agg0, _ = fused.sage2_forward(b.x, blk, "mean", params, p, 1234, None)
        res[f"{scale}_{p}"] = (h.cpu(), out.cpu(), agg0.cpu())
torch.cuda.synchronize()
torch.save(res, sys.argv[1])
print("dumped", list(res))
