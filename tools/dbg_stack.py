"""Debug helper: whole-stack fwd/bwd of ngnn.SAGE vs the oracle for a list of
(K, hidden, aggr) shapes; prints max |diff| per output / parameter gradient."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "noise-gnn_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import ngnn  # noqa: E402
from oracle import pyg_ref  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    from ngnn.loader import sample_block, synthetic_graph
    from ngnn.fused import exact_f32
    cases = [("ogbn-arxiv", 128, H, 40, "max", [15, 10], 1024, mode)
             for H in (64, 128, 192, 256) for mode in ("x3", "exact", "det")]
    cases += [("computers", 767, 512, 10, "max", [10, 5], 300, "det")]
    for name, K, H, C, aggr, fan, bs, mode in cases:
        g = synthetic_graph(name, dev, seed=0, num_features=K)
        b = sample_block(g, g.train_idx[:bs], fan, seed=5)
        torch.manual_seed(2)
        mine = ngnn.SAGE(K, H, C, 2, dropout=0.5, aggr=aggr).to(dev).eval()
        ref = pyg_ref.SAGE(K, H, C, 2, dropout=0.5, aggr=aggr).eval()
        ref.load_state_dict({k: v.cpu() for k, v in mine.state_dict().items()})
        x = b.x.clone().requires_grad_(True)
        torch.use_deterministic_algorithms(mode == "det")
        with exact_f32(mode == "exact"):
            out = mine(x, b.edge_index)
            F.cross_entropy(out[:b.batch_size], b.y[:b.batch_size]).backward()
        torch.use_deterministic_algorithms(False)
        xr = b.x.cpu().clone().requires_grad_(True)
        out_r = ref(xr, b.edge_index.cpu())
        F.cross_entropy(out_r[:b.batch_size], b.y[:b.batch_size].cpu()).backward()
        res = {"out": (out.detach().cpu() - out_r.detach()).abs().max().item(),
               "dx": (x.grad.cpu() - xr.grad).abs().max().item()}
        for (k, p), (_, q) in zip(mine.named_parameters(), ref.named_parameters()):
            d = (p.grad.cpu() - q.grad).abs()
            res[k] = (d.max().item(), q.grad.abs().max().item(), int(d.argmax()))
        print(name, K, H, aggr, mode, b.num_nodes, b.edge_index.shape[1], res, flush=True)


if __name__ == "__main__":
    main()
