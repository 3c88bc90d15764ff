"""Debug: per-conv 3-layer middle conv weight gradient vs oracle."""
import sys
sys.path.insert(0, "noise-gnn_amd"); sys.path.insert(0, "."); sys.path.insert(0, "tests")
import torch
import torch.nn.functional as F
import ngnn
from ngnn import fused
from oracle import pyg_ref
from test_gpu_perconv import _RefSAGE, _block
b = _block(fan=(10, 5, 3))
torch.manual_seed(5)
mine = _RefSAGE(ngnn.SAGEConv, 100, 64, 47, 3).to("cuda").eval()
ref = pyg_ref.SAGE(100, 64, 47, 3).eval()
ref.load_state_dict({k: v.cpu() for k, v in mine.state_dict().items()})
fused._debug_grads = []
x = b.x.clone().requires_grad_(True)
out = mine(x, b.edge_index)
F.cross_entropy(out[:b.batch_size], b.y[:b.batch_size]).backward()
torch.cuda.synchronize()
dbg = fused._debug_grads
fused._debug_grads = None
print("entries", len(dbg), [d[0] for d in dbg])
ei = b.edge_index.cpu()
src, dst = ei
N = b.num_nodes
deg = torch.bincount(dst, minlength=N)
print("N", N, "rows with in-edges", int((deg > 0).sum()), "last target", int(dst.max()))
for j, (i, dy, agg, hin) in enumerate(dbg):
    dy, agg, hin = dy.cpu(), agg.cpu(), hin.cpu()
    want = torch.zeros(N, hin.size(1)).index_add_(0, dst, hin[src]) / deg.clamp(min=1)[:, None]
    R = int((dy.abs().sum(1) > 0).nonzero().max()) + 1
    bad = (agg[:R] - want[:R]).abs().max(1).values
    print(f"entry {j} layer {i}: R={R}, agg max err rows<R {float(bad.max()):.3g} at row {int(bad.argmax())}, deg there {int(deg[int(bad.argmax())])}, n bad rows {(bad > 1e-4).sum().item()}")
# weight gradients of each conv from its own tensors (float64 on the host)
convs = list(mine.convs)[::-1]  # backward order: conv2, conv1, conv0
for j, (i, dy, agg, hin) in enumerate(dbg):
    dy, agg, hin = dy.cpu().double(), agg.cpu().double(), hin.cpu().double()
    R = int((dy.abs().sum(1) > 0).nonzero().max()) + 1
    aggm = agg[:R] * (deg[:R] > 0).double()[:, None]
    c = convs[j]
    for name, want, got in (("dWl", dy[:R].T @ aggm, c.lin_l.weight.grad),
                            ("dWr", dy.T @ hin, c.lin_r.weight.grad),
                            ("db", dy.sum(0), c.lin_l.bias.grad)):
        d = (got.cpu().double() - want).abs()
        print(f"conv{2 - j} {name}: max err {float(d.max()):.3g} / max {float(want.abs().max()):.3g}; argmax {divmod(int(d.argmax()), want.shape[-1]) if want.dim() == 2 else int(d.argmax())}")
# the oracle's output gradient of every conv (retain_grad on its outputs)
outs = []
class Hook(torch.nn.Module):
    pass
xr = b.x.cpu().clone()
h = xr
for ci, conv in enumerate(ref.convs):
    h = conv(h, ei)
    h.retain_grad()
    outs.append(h)
    if ci != 2:
        h = h.relu()
F.cross_entropy(h[:b.batch_size], b.y[:b.batch_size].cpu()).backward()
for j, (i, dy, agg, hin) in enumerate(dbg):
    ci = 2 - j
    want = outs[ci].grad
    d = (dy.cpu() - want).abs()
    rowerr = d.max(1).values
    print(f"conv{ci} dout: max err {float(d.max()):.3g} / max {float(want.abs().max()):.3g}; rows with err>1e-7: {(rowerr > 1e-7).sum().item()} first {int((rowerr > 1e-7).nonzero()[0]) if (rowerr > 1e-7).any() else -1}; nonzero rows mine {(dy.abs().sum(1) > 0).sum().item()} want {(want.abs().sum(1) > 0).sum().item()}")
# is the bad row a ReLU tie?  conv1 pre-activations where the output gradients differ
acts = {}
mine.convs[1].register_forward_hook(lambda m, a, o: acts.__setitem__("c1", o.detach().cpu()))
with torch.no_grad():
    mine(b.x.clone(), b.edge_index)
dy1 = dbg[1][1].cpu()
d = (dy1 - outs[1].grad).abs()
for r, c in (d > 1e-7).nonzero().tolist()[:10]:
    print(f"elem ({r},{c}): mine pre-act {float(acts['c1'][r, c]):.3e} ref pre-act {float(outs[1][r, c]):.3e} "
          f"dy mine {float(dy1[r, c]):.3e} ref {float(outs[1].grad[r, c]):.3e}")
