"""Round-5 diagnostic: where does dW_l0 of the eval-mode stack differ from the
oracle?  (tests/test_gpu_fwd2.py::test_fwd2_stack_backward_matches_oracle[mean-False])"""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "noise-gnn_amd"), os.path.join(os.path.dirname(__file__), ".."),
                os.path.join(os.path.dirname(__file__), "..", "tests")]
import torch, torch.nn.functional as F
import ngnn
from ngnn import fused
from ngnn.block import get_block
from oracle import pyg_ref, c_agg
from ngnn.loader import sample_block, synthetic_graph
DEV = torch.device("cuda:0")
graph = synthetic_graph("ogbn-products", DEV, seed=2, scale=0.01)
b = sample_block(graph, graph.train_idx[:256], [15, 10], seed=4)
N = b.num_nodes
ei = b.edge_index.cpu()
deg = torch.bincount(ei[1], minlength=N)
blk = get_block(b.edge_index, N)
print("N", N, "E", ei.shape[1], "n_active", blk.n_active, "rows with deg>0:", int((deg > 0).sum()),
      "max row with deg>0:", int((deg > 0).nonzero().max()), "deg0 rows below n_active:", int((deg[:blk.n_active] == 0).sum()))
src, dst = ei
Rn = max(256, int(src[dst < 256].max()) + 1)
print("R'", Rn, "deg0 rows below R'", int((deg[:Rn] == 0).sum()))
for trial in range(3):
    torch.manual_seed(11)
    mine = ngnn.SAGE(100, 256, 47, 2, dropout=0.5, aggr="mean").to(DEV).eval()
    params = [q for c in mine.convs for q in (c.lin_l.weight, c.lin_l.bias, c.lin_r.weight)]
    h, out, agg0, _ = fused.sage2_forward(b.x, blk, "mean", params, 0.0, 0, None)
    torch.cuda.synchronize()
    want = torch.from_numpy(c_agg.agg_fwd(b.x.cpu().numpy(), ei.numpy(), N, "mean"))
    a = agg0.cpu()
    has = deg > 0
    bad = (a[has] != want[has]).any(1)
    print("trial", trial, "agg0 rows with edges that differ:", int(bad.sum()), "of", int(has.sum()))
    x = b.x.clone().requires_grad_(True)
    out = mine(x, b.edge_index)
    F.cross_entropy(out[:256], b.y[:256]).backward()
    ref = pyg_ref.SAGE(100, 256, 47, 2, aggr="mean").eval()
    ref.load_state_dict({k: v.cpu() for k, v in mine.state_dict().items()})
    xr = b.x.cpu().clone().requires_grad_(True)
    out_r = ref(xr, ei)
    F.cross_entropy(out_r[:256], b.y[:256].cpu()).backward()
    for (k, p), (_, q) in zip(mine.named_parameters(), ref.named_parameters()):
        d = (p.grad.cpu() - q.grad).abs()
        print(f"  {k}: ratio {float(d.max() / q.grad.abs().max()):.2e} at {tuple(int(i) for i in (d == d.max()).nonzero()[0])}")
    # per-row attribution of dW_l0: rows whose dz0 x agg contributes the error
    g_wl0 = mine.convs[0].lin_l.weight.grad.cpu()
    dz_r = None
