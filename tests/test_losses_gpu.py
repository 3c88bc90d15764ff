"""ngnn.losses.seed_cross_entropy == F.cross_entropy(out[:B], y[:B]) (the
reference loop's loss, pipeline.py:158): value, input gradient, ignored
labels, and the SAGE backward fed by it (row-bound hint) against the same
backward fed by torch's loss."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


# B <= 4096: the one-launch forward + gradient; larger (a full-batch seed
# set): the O(B) three-launch path (the one-launch count is O(B^2))
@pytest.mark.parametrize("C,B", [(47, 256), (10, 256), (130, 256), (47, 4096), (47, 5000),
                                 (47, 100_000), (10, 200_000)])
def test_value_and_grad(C, B):
    from ngnn.losses import seed_cross_entropy
    g = torch.Generator().manual_seed(C)
    N = B + 444
    x = (torch.randn(N, C, generator=g) * 3).to(DEV).requires_grad_(True)
    y = torch.randint(0, C, (N,), generator=g).to(DEV)
    y[5] = -100  # ignored label
    x2 = x.detach().clone().requires_grad_(True)
    got = seed_cross_entropy(x, y, B)
    ref = F.cross_entropy(x2[:B], y[:B])
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)
    got.backward()
    ref.backward()
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-5, atol=1e-7)
    assert torch.count_nonzero(x.grad[B:]) == 0


def test_sage_step_same_grads_as_torch_loss():
    import ngnn
    from ngnn.losses import seed_cross_entropy
    from ngnn.loader import NeighborLoader, synthetic_graph
    gr = synthetic_graph("ogbn-arxiv", DEV, seed=0, scale=0.05)
    b = next(iter(NeighborLoader(gr, gr.train_idx, [10, 5], 256, shuffle=True, seed=3)))
    torch.manual_seed(4)
    m1 = ngnn.SAGE(gr.x.size(1), 64, gr.num_classes, 2, dropout=0.0).to(DEV)
    m2 = ngnn.SAGE(gr.x.size(1), 64, gr.num_classes, 2, dropout=0.0).to(DEV)
    m2.load_state_dict(m1.state_dict())
    seed_cross_entropy(m1(b.x, b.edge_index), b.y, b.batch_size).backward()
    F.cross_entropy(m2(b.x, b.edge_index)[:b.batch_size], b.y[:b.batch_size]).backward()
    for (n, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        torch.testing.assert_close(p1.grad, p2.grad, rtol=1e-4, atol=1e-6, msg=n)


def test_cpu_raises():
    from ngnn.losses import seed_cross_entropy
    with pytest.raises(RuntimeError):
        seed_cross_entropy(torch.zeros(4, 3), torch.zeros(4, dtype=torch.long), 2)


# ---- co-teaching loss (CTLoss, losses.py:19-49) on the device

import os  # noqa: E402

import numpy as np  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from ngnn.losses import CTLoss  # noqa: E402
from oracle import losses_ref  # noqa: E402


def _run_ct(y1, y2, yn, forget, ind, clean):
    a = y1.cuda().requires_grad_(True)
    b = y2.cuda().requires_grad_(True)
    out = CTLoss("cuda")(a, b, yn.cuda(), forget, None if ind is None else ind.cuda(),
                         None if clean is None else clean.cuda())
    out[0].backward()
    out[1].backward()
    return out, a.grad, b.grad


@pytest.mark.parametrize("name", ["ct_loss_b300", "ct_loss_b1024"])
def test_ct_loss_vs_reference_fixture(golden_dir, name):
    g = np.load(os.path.join(golden_dir, name + ".npz"))
    y1, y2 = torch.from_numpy(g["y1"]), torch.from_numpy(g["y2"])
    yn = torch.from_numpy(g["y_noise"])
    (l1, l2, p1, p2, i1, i2, n1, n2), g1, g2 = _run_ct(
        y1, y2, yn, float(g["forget_rate"]), torch.from_numpy(g["ind"]),
        torch.from_numpy(g["noise_or_not"]))
    R = len(g["ind_1_update"])
    assert i1.numel() == R and n1.numel() == len(y1) - R
    for m, (y, ik, nk, dev_sorted) in enumerate(((y1, "ind_1_update", "ind_noisy_1", torch.cat([i1, n1])),
                                                 (y2, "ind_2_update", "ind_noisy_2", torch.cat([i2, n2])))):
        lref = F.cross_entropy(y, yn, reduction="none")
        ref_sorted = torch.from_numpy(np.concatenate([g[ik], g[nk]]))
        # a valid ascending order of the same losses (fp32 row losses may differ by an ulp,
        # so near-ties may swap); identical positions wherever the gap is clear
        torch.testing.assert_close(lref[dev_sorted.cpu()], lref[ref_sorted], rtol=0, atol=2e-6)
        gap = (lref[ref_sorted][R] - lref[ref_sorted][R - 1]).item()
        if gap > 1e-5:
            assert set(dev_sorted[:R].tolist()) == set(ref_sorted[:R].tolist())
    torch.testing.assert_close(l1.detach().cpu(), torch.from_numpy(g["loss_1"]), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(l2.detach().cpu(), torch.from_numpy(g["loss_2"]), rtol=1e-5, atol=1e-6)
    assert abs(float(p1) - float(g["pure_ratio_1"])) < 1e-6
    assert abs(float(p2) - float(g["pure_ratio_2"])) < 1e-6
    torch.testing.assert_close(g1.cpu(), torch.from_numpy(g["grad_y1"]), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(g2.cpu(), torch.from_numpy(g["grad_y2"]), rtol=1e-5, atol=1e-7)


def _separated_logits(B, C, seed):
    """rows whose losses are far apart (well-defined order): label 0, other
    logits 0, the first logit stepping evenly over [-3, 3] in shuffled row
    order (loss strictly monotone in it; gaps >= ~4e-4 at B = 8192)"""
    gen = torch.Generator().manual_seed(seed)
    y = torch.zeros(B, C)
    y[:, 0] = torch.linspace(-3, 3, B)[torch.randperm(B, generator=gen)]
    return y


@pytest.mark.parametrize("B,C,forget", [(1024, 47, 0.2), (17, 3, 0.5), (4096, 10, 0.0),
                                        (8192, 40, 0.9), (5, 2, 1.0)])
def test_ct_loss_vs_oracle_separated(B, C, forget):
    y1, y2 = _separated_logits(B, C, 1), _separated_logits(B, C, 2)
    yn = torch.zeros(B, dtype=torch.long)
    ind = torch.randperm(3 * B)[:B]
    clean = torch.rand(3 * B) < 0.5
    dev_out, g1, g2 = _run_ct(y1, y2, yn, forget, ind, clean)
    a, b = y1.clone().requires_grad_(True), y2.clone().requires_grad_(True)
    ref = losses_ref.ct_loss(a, b, yn, forget, ind, clean)
    R = ref[4].numel()
    for k in (4, 5, 6, 7):  # index outputs: bitwise
        assert torch.equal(dev_out[k].cpu(), ref[k]), k
    if R == 0:  # empty selection: NaN, as torch's mean of nothing
        assert torch.isnan(dev_out[0]).item() and torch.isnan(dev_out[2]).item()
        return
    for k in (0, 1, 2, 3):
        torch.testing.assert_close(dev_out[k].detach().cpu().float(), ref[k].detach().float(),
                                   rtol=1e-5, atol=1e-6)
    ref[0].backward()
    ref[1].backward()
    torch.testing.assert_close(g1.cpu(), a.grad, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(g2.cpu(), b.grad, rtol=1e-5, atol=1e-7)


def test_ct_loss_ties_and_ignore_index():
    B, C = 64, 5
    y1 = torch.zeros(B, C)  # every loss ties: order by row index
    y2 = _separated_logits(B, C, 3)
    yn = torch.zeros(B, dtype=torch.long)
    yn[::7] = -100  # ignored rows: loss 0 -> sorted first, excluded from the means
    dev_out, g1, g2 = _run_ct(y1, y2, yn, 0.25, None, torch.ones(B, dtype=torch.bool))
    a, b = y1.clone().requires_grad_(True), y2.clone().requires_grad_(True)
    ref = losses_ref.ct_loss(a, b, yn, 0.25, torch.arange(B), torch.ones(B, dtype=torch.bool))
    for k in (4, 5, 6, 7):
        assert torch.equal(dev_out[k].cpu(), ref[k]), k
    for k in (0, 1, 2, 3):
        torch.testing.assert_close(dev_out[k].detach().cpu().float(), ref[k].detach().float(),
                                   rtol=1e-5, atol=1e-6)
    ref[0].backward()
    ref[1].backward()
    torch.testing.assert_close(g1.cpu(), a.grad, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(g2.cpu(), b.grad, rtol=1e-5, atol=1e-7)


def test_ct_loss_backwards_are_independent():
    """loss_1.backward() touches only model 1's graph (pipeline.py:125-131)."""
    w1 = torch.randn(8, 4, device="cuda", requires_grad=True)
    w2 = torch.randn(8, 4, device="cuda", requires_grad=True)
    x = torch.randn(32, 8, device="cuda")
    out = CTLoss("cuda")(x @ w1, x @ w2, torch.randint(0, 4, (32,), device="cuda"), 0.3, None, None)
    out[0].backward()
    assert w1.grad is not None and w2.grad is None
    out[1].backward()
    assert w2.grad is not None


def test_bf16_logits_seed_rows_only():
    """bf16 logits: only the seed rows are widened; value equals
    F.cross_entropy on the widened rows, the gradient is bf16 with rows >= B
    exactly zero and carries the row hint; the bf16 stack output (one cast
    launch) equals Tensor.to(bfloat16) bitwise."""
    from ngnn.fused import _StackOutBF16
    from ngnn.losses import seed_cross_entropy
    g = torch.Generator().manual_seed(3)
    N, C, B = 3000, 47, 512
    xf = (torch.randn(N, C, generator=g) * 4).to(DEV)
    xf[7, 3] = float("nan")
    xf[8, 1] = float("inf")
    xb = _StackOutBF16.apply(xf)
    assert torch.equal(xb.view(torch.int16), xf.to(torch.bfloat16).view(torch.int16))
    x = (torch.randn(N, C, generator=g) * 3).to(DEV).to(torch.bfloat16).requires_grad_(True)
    y = torch.randint(0, C, (N,), generator=g).to(DEV)
    got = seed_cross_entropy(x, y, B)
    x2 = x.detach().float().requires_grad_(True)
    ref = F.cross_entropy(x2[:B], y[:B])
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)
    got.backward()
    ref.backward()
    assert x.grad.dtype == torch.bfloat16
    assert torch.equal(x.grad[B:], torch.zeros_like(x.grad[B:]))
    # (fp32 gradients equal to ~1 ulp, then each rounded to bf16: <= 1 bf16 ulp apart)
    torch.testing.assert_close(x.grad.float(), x2.grad.to(torch.bfloat16).float(), rtol=8e-3, atol=1e-7)
