"""The co-teaching training step (pipeline.py:95-142, ``train_ct``: what
config_products.yml / config_amazon.yml run, ``algo_type: 'coteaching'``)
through ngnn.graphs.GraphedCoTeachingStep -- both SAGE models, CTLoss, both
backwards and both Adam steps as one HIP-graph replay -- against the CPU
oracle: oracle/pyg_ref.py for the two models (the replay's dropout masks
rebuilt from the slot seed, model 2 salted) and oracle/losses_ref.py for
CTLoss (the reference's losses.py:19-49 restated; pinned bitwise against the
reference's own CTLoss by tests/golden/ct_loss_*.npz).

Bars: losses 1e-5; pure ratios exact; the kept / forgotten row sets equal
(rows whose losses lie within 1e-5 of the selection boundary may swap: fp32
summation order decides them -- the oracle then takes the GPU's selection,
as _MaskedSAGE takes its ReLU kinks); every weight gradient of both models
at the fp32 bar (tests/gradbar.py); post-step parameters as torch's Adam."""
import pytest
import torch
import torch.nn.functional as F

import ngnn
from oracle.losses_ref import ct_loss

from gradbar import assert_wgrad
from test_gpu_fused import _MaskedSAGE, dropout_keep

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _selection(loss, nr, got_sel, tol=1e-5):
    """The oracle's kept set of one model, given its per-row losses: the nr
    smallest (stable), except that rows within tol of the boundary loss may
    be swapped for the GPU's choice (got_sel)."""
    order = torch.sort(loss, stable=True).indices
    mine = set(order[:nr].tolist())
    got = set(got_sel.tolist())
    if mine == got:
        return order[:nr]
    bound = float(loss[order[nr - 1]])
    for r in mine ^ got:
        assert abs(float(loss[r]) - bound) <= tol * max(1.0, abs(bound)), \
            f"row {r}: loss {float(loss[r])} vs boundary {bound} -- not a near tie"
    return got_sel.cpu()


@pytest.mark.timeout(400)
@pytest.mark.parametrize("forget_rate", [0.2, 0.0])
def test_coteaching_graph_step_full_products_block(forget_rate):
    from ngnn import fused
    from ngnn.graphs import GraphedCoTeachingStep, slot_size
    from ngnn.loader import sample_block, synthetic_graph
    from ngnn.losses import CTLoss
    from ngnn.optim import Adam
    g = synthetic_graph("ogbn-products", DEV, seed=0)
    # noisy labels (flip_label's role, pipeline.py:72): 30 % of the nodes
    # relabelled uniformly; noise_or_not = label kept
    gen = torch.Generator(device=DEV).manual_seed(5)
    flip = torch.rand(g.num_nodes, device=DEV, generator=gen) < 0.3
    yhn = torch.where(flip, torch.randint(0, 47, (g.num_nodes,), device=DEV, generator=gen), g.y)
    noise_or_not = yhn == g.y
    b = sample_block(g, g.train_idx[:1024], [15, 10], seed=21)
    warm = sample_block(g, g.train_idx[1024:2048], [15, 10], seed=22)
    N = b.num_nodes
    yb, yw = yhn[b.n_id], yhn[warm.n_id]
    torch.manual_seed(11)
    m1 = ngnn.SAGE(100, 256, 47, 2, dropout=0.5).to(DEV).train()
    m2 = ngnn.SAGE(100, 256, 47, 2, dropout=0.5).to(DEV).train()
    init = [{k: v.detach().cpu().clone() for k, v in m.state_dict().items()} for m in (m1, m2)]
    o1, o2 = Adam(m1.parameters(), lr=1e-3), Adam(m2.parameters(), lr=1e-3)
    n_cap, e_cap = slot_size(1024, [15, 10])
    step = GraphedCoTeachingStep(m1, o1, m2, o2, CTLoss(DEV), 1024, n_cap, e_cap, 100, DEV,
                                 noise_or_not=noise_or_not)
    fused._debug_acts = []
    try:
        step.capture(warm.x, warm.edge_index, yw, warm.n_id, forget_rate)
        acts = fused._debug_acts[-2:]  # (the captured forwards' hidden activations)
    finally:
        fused._debug_acts = None
    l1, l2, pr1, pr2, k1, k2, f1, f2 = step(b.x, b.edge_index, yb, b.n_id, forget_rate)
    torch.cuda.synchronize()
    assert step.zero_copy
    nr = step.num_remember(forget_rate)
    assert k1.numel() == nr and f1.numel() == 1024 - nr
    seed_state = int(step.seed_state.item()) & (2**64 - 1)
    rn = int(step.r_next.item()) & 0xFFFFFFFF
    x, ei = b.x.cpu(), b.edge_index.cpu()
    outs, refs = [], []
    for mi, (m, salt) in enumerate(((m1, 0), (m2, m2._ngnn_graph_salt))):
        masks = [dropout_keep((salt + 7919 * i) ^ seed_state, N, 256, 0.5).float() for i in range(1)]
        ref = _MaskedSAGE(100, 256, 47, 2, dropout=0.5, masks=masks,
                          gpu_hidden=[a.cpu() for a in acts[mi]], kink_rows=rn)
        ref.load_state_dict(init[mi])
        refs.append(ref)
        outs.append(ref(x, ei))
    ys = yb[:1024].cpu()
    # the selections: each model's own per-row losses decide what the OTHER is trained on
    ce = [F.cross_entropy(o[:1024].detach(), ys, reduction="none") for o in outs]
    sel1 = _selection(ce[0], nr, k1) if nr else k1.cpu()
    sel2 = _selection(ce[1], nr, k2) if nr else k2.cpu()
    ref_out = ct_loss(outs[0][:1024], outs[1][:1024], ys, forget_rate, b.n_id[:1024].cpu(),
                      noise_or_not.cpu())
    if torch.equal(ref_out[4].sort().values, sel1.sort().values) and \
            torch.equal(ref_out[5].sort().values, sel2.sort().values):
        lr1, lr2, prr1, prr2 = ref_out[:4]
    else:  # a boundary near tie: the exchange on the GPU's selection
        lr1 = F.cross_entropy(outs[0][:1024][sel2], ys[sel2])
        lr2 = F.cross_entropy(outs[1][:1024][sel1], ys[sel1])
        nn_ = noise_or_not.cpu()[b.n_id[:1024].cpu()]
        prr1, prr2 = nn_[sel1].sum() / float(nr), nn_[sel2].sum() / float(nr)
    assert abs(float(l1) - float(lr1)) < 1e-5 and abs(float(l2) - float(lr2)) < 1e-5
    assert float(pr1) == pytest.approx(float(prr1), abs=1e-7)
    assert float(pr2) == pytest.approx(float(prr2), abs=1e-7)
    assert set(k1.tolist()).isdisjoint(f1.tolist()) and set(k2.tolist()).isdisjoint(f2.tolist())
    lr1.backward()
    lr2.backward()
    for mi, (m, ref) in enumerate(((m1, refs[0]), (m2, refs[1]))):
        for k, q in ref.named_parameters():
            p = dict(m.named_parameters())[k]
            assert_wgrad(p.grad.detach().cpu(), q.grad, msg=f"model{mi + 1}:{k}")
        o_ref = torch.optim.Adam(ref.parameters(), lr=1e-3)
        o_ref.step()
        for k, q in ref.named_parameters():
            p = dict(m.named_parameters())[k].detach().cpu()
            sure = q.grad.abs() > 1e-4
            torch.testing.assert_close(p[sure], q.detach()[sure], rtol=0, atol=2e-6, msg=f"model{mi + 1}:{k}")
    # the kink overrides stay a handful
    for ref in refs:
        assert sum(ref.kinks) <= 64, ref.kinks


def test_coteaching_short_block_runs_eagerly():
    """An epoch's last block (batch_size < the captured B) takes the same
    loop body eagerly: num_remember of its own size, finite losses."""
    from ngnn.graphs import GraphedCoTeachingStep, slot_size
    from ngnn.loader import sample_block, synthetic_graph
    from ngnn.losses import CTLoss
    from ngnn.optim import Adam
    g = synthetic_graph("ogbn-products", DEV, seed=1, scale=0.01)
    torch.manual_seed(3)
    m1 = ngnn.SAGE(100, 64, 47, 2).to(DEV).train()
    m2 = ngnn.SAGE(100, 64, 47, 2).to(DEV).train()
    n_cap, e_cap = slot_size(256, [5, 4])
    step = GraphedCoTeachingStep(m1, Adam(m1.parameters()), m2, Adam(m2.parameters()), CTLoss(DEV), 256,
                                 n_cap, e_cap, 100, DEV, noise_or_not=torch.ones(g.num_nodes, dtype=torch.bool,
                                                                                 device=DEV))
    full = sample_block(g, g.train_idx[:256], [5, 4], seed=1)
    short = sample_block(g, g.train_idx[256:356], [5, 4], seed=2)
    out = step(full.x, full.edge_index, g.y[full.n_id], full.n_id, 0.25)
    assert out[4].numel() == 192
    out = step(short.x, short.edge_index, g.y[short.n_id], short.n_id, 0.25, batch_size=100)
    torch.cuda.synchronize()
    assert out[4].numel() == 75 and out[6].numel() == 25
    assert torch.isfinite(out[0]) and torch.isfinite(out[1]) and float(out[2]) == 1.0
