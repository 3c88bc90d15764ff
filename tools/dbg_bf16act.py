"""Debug: a small bf16 SAGE stack with bf16 hidden activations vs the same
stack with fp32 activations (out_bf16 forced off): per-parameter gradient
differences."""
import sys
sys.path.insert(0, "noise-gnn_amd"); sys.path.insert(0, ".")
import torch
import torch.nn.functional as F
import ngnn
from ngnn import fused
from ngnn.loader import sample_block, synthetic_graph
DEV = "cuda"
g = synthetic_graph("ogbn-products", DEV, seed=3, scale=0.01)
g.x = g.x.to(torch.bfloat16)
b = sample_block(g, g.train_idx[:512], [10, 8, 5], seed=2)
torch.manual_seed(5)
m = ngnn.SAGE(100, 256, 47, 3, dropout=0.0).to(DEV).to(torch.bfloat16).eval()
orig = fused.sage_layer_fwd
res = {}
for mode in ("bf16act", "f32act"):
    if mode == "f32act":
        def patched(*a, **k):
            want = k.get("out_bf16", False)
            k["out_bf16"] = False
            h = orig(*a, **k)
            return h.bfloat16().float() if want else h  # the same values, fp32 rows
        fused.sage_layer_fwd = patched
    m.zero_grad(set_to_none=True)
    out = m(b.x, b.edge_index)
    loss = F.cross_entropy(out[:512].float(), b.y[:512])
    loss.backward()
    torch.cuda.synchronize()
    res[mode] = (out.detach().float().cpu(), float(loss),
                 {k: p.grad.detach().float().cpu().clone() for k, p in m.named_parameters()})
fused.sage_layer_fwd = orig
o1, l1, g1 = res["bf16act"]
o2, l2, g2 = res["f32act"]
print("logits max diff", float((o1 - o2).abs().max()), "max", float(o2.abs().max()), "loss", l1, l2)
for k in g1:
    d = (g1[k] - g2[k]).abs()
    print(f"{k}: max diff {float(d.max()):.3g} / max {float(g2[k].abs().max()):.3g}")
