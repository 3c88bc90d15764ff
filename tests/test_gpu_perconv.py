"""INTEGRATION.md option A: the reference's own wrapper structure (sage.py:6-40,
convolution.py:7-35 -- conv, relu, F.dropout per layer, logits last) with
ngnn.SAGEConv / ngnn.GCNConv swapped in for PyG's, as `from ngnn import
SAGEConv` in place of sage.py:4 would do.  Forward and backward (every
parameter gradient and the input gradient) against the oracle, and the
training step issues no library GEMM: torch's matmul entry points are
patched to raise for the duration of the step.
"""
from unittest import mock

import pytest
import torch
import torch.nn.functional as F

import ngnn
from oracle import pyg_ref

from test_gpu_fused import GRAD, OUT
from gradbar import assert_wgrad

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


class _RefSAGE(torch.nn.Module):
    """sage.py:6-40's structure over a given conv class (use_bn False)."""

    def __init__(self, conv, in_size, hidden, out, num_layers, dropout=0.5, aggr="mean"):
        super().__init__()
        self.num_layers, self.dropout = num_layers, dropout
        dims = [in_size] + [hidden] * (num_layers - 1) + [out]
        self.convs = torch.nn.ModuleList(conv(dims[i], dims[i + 1], aggr=aggr)
                                         for i in range(num_layers))

    def forward(self, x, edge_index):
        for i, conv in enumerate(self.convs):
            x = conv(x, edge_index)
            if i != self.num_layers - 1:
                x = F.relu(x)
                x = F.dropout(x, p=self.dropout, training=self.training)
        return x


class _RefGCN(torch.nn.Module):
    """convolution.py:7-35's structure over a given conv class."""

    def __init__(self, conv, in_size, hidden, out, num_layers, dropout=0.5):
        super().__init__()
        self.num_layers, self.dropout = num_layers, dropout
        dims = [in_size] + [hidden] * (num_layers - 1) + [out]
        self.convs = torch.nn.ModuleList(conv(dims[i], dims[i + 1], normalize=False)
                                         for i in range(num_layers))

    def forward(self, x, edge_index):
        for i, conv in enumerate(self.convs):
            x = conv(x, edge_index)
            if i != self.num_layers - 1:
                x = F.relu(x)
                x = F.dropout(x, p=self.dropout, training=self.training)
        return x


def _no_gemm():
    """Patches torch's GEMM entry points (F.linear, matmul, mm, addmm, bmm) to
    raise: a step that reaches rocBLAS / hipBLASLt through them fails."""
    def boom(*a, **k):
        raise AssertionError("library GEMM called on the per-conv path")
    return [mock.patch.object(F, "linear", boom), mock.patch.object(torch, "matmul", boom),
            mock.patch.object(torch, "mm", boom), mock.patch.object(torch, "addmm", boom),
            mock.patch.object(torch, "bmm", boom)]


def _block(seed=3, scale=0.01, fan=(10, 5), bs=256):
    from ngnn.loader import sample_block, synthetic_graph
    g = synthetic_graph("ogbn-products", DEV, seed=seed, scale=scale)
    return sample_block(g, g.train_idx[:bs], list(fan), seed=seed + 1)


def _tie_sync(mine, ref):
    """Hooks making the wrapper's ReLU see the same sign on both sides where
    a conv output is within fp32 rounding of zero (|v| < 1e-6): there the two
    summation orders may disagree on the sign (observed: -7.5e-8 vs +6.0e-8),
    and the ReLU mask -- not the kernels -- would then decide a gradient
    element.  The reference's output takes the kernel's value at such
    elements as a constant offset, so its gradients are unchanged."""
    seen = []
    hooks = [c.register_forward_hook(lambda m, a, o: seen.append(o.detach().float().cpu()))
             for c in mine.convs]

    def sync(m, a, o):
        k = seen[ref_i[0]]
        ref_i[0] += 1
        tie = (o.abs() < 1e-6) & ((o > 0) != (k > 0))
        return o + torch.where(tie, k - o, torch.zeros_like(o)).detach()
    ref_i = [0]
    return seen, hooks, [c.register_forward_hook(sync) for c in ref.convs]


def _compare(mine, ref, b, dtype=torch.float32, tol_out=OUT, tol_g=GRAD, tol_w=None):
    x = b.x.to(dtype).clone().requires_grad_(True)
    patches = _no_gemm()
    _, mh, rh = _tie_sync(mine, ref)
    for p in patches:
        p.start()
    try:
        out = mine(x, b.edge_index)
        loss = F.cross_entropy(out[:b.batch_size].float(), b.y[:b.batch_size])
        loss.backward()
        torch.cuda.synchronize()
    finally:
        for p in patches:
            p.stop()
        for h in mh:
            h.remove()
    xr = b.x.to(dtype).float().cpu().clone().requires_grad_(True)
    try:
        out_r = ref(xr, b.edge_index.cpu())
    finally:
        for h in rh:
            h.remove()
    F.cross_entropy(out_r[:b.batch_size], b.y[:b.batch_size].cpu()).backward()
    torch.testing.assert_close(out.detach().float().cpu(), out_r.detach(), **tol_out)
    torch.testing.assert_close(x.grad.float().cpu(), xr.grad, **tol_g)
    for (k, p), (_, q) in zip(mine.named_parameters(), ref.named_parameters()):
        if tol_w is None:
            assert_wgrad(p.grad.float().cpu(), q.grad, msg=k)
            continue
        d = (p.grad.float().cpu() - q.grad).abs()
        torch.testing.assert_close(p.grad.float().cpu(), q.grad, **tol_w,
                                   msg=f"{k}: max |diff| {d.max():.3g} (|ref| max {q.grad.abs().max():.3g})")


@pytest.mark.parametrize("layers,aggr", [(2, "mean"), (3, "mean"), (2, "max"), (2, "sum")])
def test_reference_wrapper_with_ngnn_sageconv(layers, aggr):
    b = _block(fan=(10, 5, 3)[:layers])
    torch.manual_seed(5)
    mine = _RefSAGE(ngnn.SAGEConv, 100, 64, 47, layers, aggr=aggr).to(DEV).eval()
    ref = pyg_ref.SAGE(100, 64, 47, layers, aggr=aggr).eval()
    ref.load_state_dict({k: v.cpu() for k, v in mine.state_dict().items()})
    # the input gradient crosses `layers` input-gradient kernels (atomic
    # scatters, fp32 summation order): atol 1e-5 per layer
    _compare(mine, ref, b, tol_g=dict(rtol=1e-4, atol=1e-5 * layers))


def test_reference_wrapper_with_ngnn_gcnconv():
    b = _block()
    torch.manual_seed(6)
    mine = _RefGCN(ngnn.GCNConv, 100, 64, 47, 2).to(DEV).eval()
    ref = pyg_ref.SimpleGCN(100, 64, 47, 2).eval()
    ref.load_state_dict({k: v.cpu() for k, v in mine.state_dict().items()})
    _compare(mine, ref, b)


def test_reference_wrapper_bf16_ngnn_sageconv():
    """A bf16 model through the per-conv path: bf16 storage, fp32 kernels,
    against the fp32 oracle at the bf16 tolerance."""
    b = _block()
    torch.manual_seed(7)
    mine = _RefSAGE(ngnn.SAGEConv, 100, 64, 47, 2).to(DEV).to(torch.bfloat16).eval()
    ref = pyg_ref.SAGE(100, 64, 47, 2).eval()
    ref.load_state_dict({k: v.float().cpu() for k, v in mine.state_dict().items()})
    bf = dict(rtol=2e-2, atol=2e-2)
    _compare(mine, ref, b, dtype=torch.bfloat16, tol_out=bf, tol_g=bf, tol_w=bf)


def test_reference_wrapper_trains_with_torch_dropout():
    """Train mode: the wrapper's own F.dropout between convs (torch's RNG);
    the step runs without library GEMMs and an optimiser step changes the
    parameters; the same step in eval mode equals the oracle (above)."""
    b = _block()
    torch.manual_seed(8)
    mine = _RefSAGE(ngnn.SAGEConv, 100, 64, 47, 2).to(DEV).train()
    opt = torch.optim.Adam(mine.parameters(), lr=1e-2)
    before = [p.detach().clone() for p in mine.parameters()]
    patches = _no_gemm()
    for p in patches:
        p.start()
    try:
        for _ in range(3):
            opt.zero_grad(set_to_none=True)
            out = mine(b.x, b.edge_index)
            F.cross_entropy(out[:b.batch_size], b.y[:b.batch_size]).backward()
            opt.step()
        torch.cuda.synchronize()
    finally:
        for p in patches:
            p.stop()
    assert all(not torch.equal(a, p.detach()) for a, p in zip(before, mine.parameters()))
    assert all(torch.isfinite(p).all() for p in mine.parameters())
