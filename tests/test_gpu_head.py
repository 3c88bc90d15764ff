"""GPU parity of the loss head (include/ngnn.h ngnn_xent_head, ABI 15): the
training step's seed-row cross entropy -- F.cross_entropy(out[:B], y[:B]) of
the reference's loop (pipeline.py:155-158) -- taken by ngnn_sage2_fwd's
narrow launch from the logits it finishes, with the gradient rows and their
scatter onto the source rows (the first step of the backward).

* loss, count, dy (rows < B) and g (rows < R') against float64 torch on the
  same logits: ignored labels, rows < B without in-edges, mean and sum; the
  logits themselves bitwise those of the head-less forward;
* g rows < R' are rewritten every call (stale contents do not leak), rows of
  dy >= B stay zero; all labels ignored -> NaN loss (0 / 0, as torch), an
  out-of-range label -> NaN;
* the graph slot's step takes it (spy) and matches the step without it:
  loss, logits, every gradient and the post-step parameters; a non-unit
  loss gradient (eager, on the slot's block) falls back to the scaled rows.
Bars: the loss and dy at 1e-6 relative (the head reduces in another order
than torch's log_softmax), g and gradients at
tests/gradbar.py's bar (1e-5 of each tensor's max).
"""
import pytest
import torch
import torch.nn.functional as F

import ngnn
from ngnn import fused, losses
from ngnn.block import Block

from gradbar import assert_wgrad

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _case(seed, N, B, Rn, F1=47, deg_max=15, ignore_every=0):
    """Target-sorted edges into rows < Rn (some rows without); the sources
    of edges into rows < B below Rn (the slot's R'), the others anywhere."""
    g = torch.Generator().manual_seed(seed)
    deg = torch.randint(0, deg_max + 1, (Rn,), generator=g)
    deg[::9] = 0
    dst = torch.repeat_interleave(torch.arange(Rn), deg)
    src = torch.where(dst < B, torch.randint(0, Rn, (dst.numel(),), generator=g),
                      torch.randint(0, N, (dst.numel(),), generator=g))
    ei = torch.stack([src, dst])
    blk = Block(ei.to(DEV), N)
    blk.n_active = Rn
    y = torch.randint(0, F1, (B,), generator=g)
    if ignore_every:
        y[::ignore_every] = -100
    return ei, blk, y


def _params(K0, F1, seed):
    torch.manual_seed(seed)
    m = ngnn.SAGE(K0, 256, F1, 2, dropout=0.5).to(DEV)
    c0, c1 = m.convs
    return [q.detach() for q in (c0.lin_l.weight, c0.lin_l.bias, c0.lin_r.weight,
                                 c1.lin_l.weight, c1.lin_l.bias, c1.lin_r.weight)]


def _forward(x, blk, reduce, params, head=None):
    h, out, agg0, _ = fused.sage2_forward(x, blk, reduce, params, 0.5, 4242, None, head=head)
    torch.cuda.synchronize()
    return out


def _reference(out, y, ei, B, reduce, Rn, F1):
    """float64 torch: the mean cross entropy over rows < B, its gradient,
    and the gradient scattered onto the sources (/ deg for mean)."""
    lg = out[:B].detach().double().requires_grad_(True)
    loss = F.cross_entropy(lg, y.to(DEV), ignore_index=-100)
    loss.backward()
    dy = lg.grad
    src, dst = ei[0].to(DEV), ei[1].to(DEV)
    deg = torch.bincount(dst, minlength=out.size(0)).double()
    m = dst < B
    w = dy[dst[m]] / (deg[dst[m]][:, None] if reduce == "mean" else 1.0)
    g = torch.zeros(Rn, F1, dtype=torch.float64, device=DEV)
    g.index_add_(0, src[m], w)
    return loss.detach(), dy, g


@pytest.mark.parametrize("reduce", ["mean", "sum"])
@pytest.mark.parametrize("K0,F1,B", [(100, 47, 300), (128, 40, 1024), (100, 33, 17)])
def test_head_matches_torch(reduce, K0, F1, B):
    N, Rn = 4000, 1800
    ei, blk, y = _case(K0 + B, N, B, Rn, F1, ignore_every=13)
    x = torch.randn(N, K0, device=DEV)
    params = _params(K0, F1, 3)
    plain = _forward(x, blk, reduce, params)
    y_dev = y.to(DEV)
    rword = torch.tensor([Rn], dtype=torch.int32, device=DEV)
    lh = fused.LossHead(y_dev, B, N, F1, rword)
    lh.g.fill_(7.0)  # stale rows: rows < R' are rewritten by the call
    lh.dy.fill_(0.0)
    res = lh.start()
    out = _forward(x, blk, reduce, params, head=res)
    assert torch.equal(out, plain), "the head changed the logits"
    loss_r, dy_r, g_r = _reference(out, y, ei, B, reduce, Rn, F1)
    assert abs(float(res.loss) - float(loss_r)) <= 1e-6 * max(1.0, abs(float(loss_r)))
    assert float(res.count) == float((y != -100).sum())
    torch.testing.assert_close(lh.dy[:B].double(), dy_r, rtol=1e-5, atol=1e-7)
    assert int(lh.dy[B:].count_nonzero()) == 0
    assert_wgrad(lh.g[:Rn, :F1].double(), g_r)
    assert int(lh.g[:Rn, F1:].count_nonzero()) == 0
    assert bool((lh.g[Rn:] == 7.0).all())  # rows past R' untouched
    # the hand-off ticket is zero again: a second call repeats the loss bitwise.
    # ABI 17: each call counts its seed edges per source into the array the
    # previous call's head did not read (single-edge sources take a plain row
    # store) -- g at the bar on every call, alternating between two blocks
    # with different sources (a count array reused after another block's
    # counts must have been cleared: a stale 1 would drop a contribution)
    ei2, blk2, _ = _case(K0 + B + 1, N, B, Rn, F1)
    g_r2 = _reference(_forward(x, blk2, reduce, params), y, ei2, B, reduce, Rn, F1)[2]
    for i in range(4):
        lh.g.fill_(7.0)
        res2 = lh.start()
        b_i, g_i = (blk2, g_r2) if i % 2 == 0 else (blk, g_r)
        _forward(x, b_i, reduce, params, head=res2)
        if i % 2 == 1:
            assert float(res2.loss) == float(res.loss)
        assert_wgrad(lh.g[:Rn, :F1].double(), g_i, msg=f"call {i + 2}")
    assert int(lh.src_count[-1]) == 1  # five calls: the selector flipped each time
    # both count paths were taken: sources with one seed edge and with several
    m = ei[1] < B
    cnt = torch.bincount(ei[0][m], minlength=Rn)
    assert int((cnt == 1).sum()) > 0 and int((cnt > 1).sum()) > 0


def test_head_ignored_and_bad_labels():
    N, Rn, B, K0, F1 = 1500, 700, 64, 100, 47
    ei, blk, y = _case(5, N, B, Rn)
    x = torch.randn(N, K0, device=DEV)
    params = _params(K0, F1, 4)
    rword = torch.tensor([Rn], dtype=torch.int32, device=DEV)
    # every label ignored: 0 / 0 = NaN (torch's empty mean), zero gradient
    yi = torch.full((B,), -100, dtype=torch.int64, device=DEV)
    lh = fused.LossHead(yi, B, N, F1, rword)
    res = lh.start()
    _forward(x, blk, "mean", params, head=res)
    assert torch.isnan(res.loss) and float(res.count) == 0.0
    assert int(lh.dy.count_nonzero()) == 0 and int(lh.g[:Rn].count_nonzero()) == 0
    # an out-of-range label: NaN loss (no out-of-bounds read), as the loss kernels
    yb = y.to(DEV).clone()
    yb[5] = 47
    lh2 = fused.LossHead(yb, B, N, F1, rword)
    res2 = lh2.start()
    _forward(x, blk, "mean", params, head=res2)
    assert torch.isnan(res2.loss)


def _graph_step(head: bool):
    from ngnn.graphs import GraphedTrainStep, slot_size
    from ngnn.loader import sample_block, synthetic_graph
    from ngnn.optim import Adam
    torch.manual_seed(0)
    graph = synthetic_graph("ogbn-products", DEV, seed=5, scale=0.02)
    b = sample_block(graph, graph.train_idx[:512], [15, 10], seed=9)
    b2 = sample_block(graph, graph.train_idx[512:1024], [15, 10], seed=10)
    torch.manual_seed(0)
    model = ngnn.SAGE(100, 256, 47, 2, dropout=0.5).to(DEV).train()
    opt = Adam(model.parameters(), lr=1e-3)
    n_cap, e_cap = slot_size(512, [15, 10])
    calls = []
    orig_ok, orig_apply = fused.head_ok, losses._HeadXent.apply

    def spy(*a):
        calls.append(1)
        return orig_apply(*a)

    fused.head_ok = orig_ok if head else (lambda *a: False)
    losses._HeadXent.apply = spy
    try:
        step = GraphedTrainStep(model, opt, 512, n_cap, e_cap, 100, DEV)
        step.capture(b2.x, b2.edge_index, b2.y)
        loss = step(b.x, b.edge_index, b.y)
        torch.cuda.synchronize()
        rec = dict(loss=float(loss), out=step.out[:b.num_nodes].detach().clone(),
                   grads={k: p.grad.detach().clone() for k, p in model.named_parameters()},
                   params={k: p.detach().clone() for k, p in model.named_parameters()})
        # eager, on the slot's block: a non-unit loss gradient (the scaled rows)
        opt.zero_grad(set_to_none=False)
        out = model(step.x, step.ei)
        (3.0 * losses.seed_cross_entropy(out, step.y, step.B)).backward()
        torch.cuda.synchronize()
        rec["grads3"] = {k: p.grad.detach().clone() for k, p in model.named_parameters()}
    finally:
        fused.head_ok, losses._HeadXent.apply = orig_ok, orig_apply
    return rec, len(calls)


def test_graph_step_takes_the_head_and_matches():
    with_head, n_with = _graph_step(True)
    without, n_without = _graph_step(False)
    assert n_with >= 2 and n_without == 0  # the captured step (and the eager call) took it
    assert abs(with_head["loss"] - without["loss"]) <= 1e-6 * max(1.0, abs(without["loss"]))
    torch.testing.assert_close(with_head["out"], without["out"], rtol=0, atol=0)
    for k in without["grads"]:
        assert_wgrad(with_head["grads"][k], without["grads"][k], msg=k)
        assert_wgrad(with_head["grads3"][k], without["grads3"][k], msg=k)
        # post-step parameters: at step 1 Adam's update is lr g / (|g| + eps),
        # compared where |g| is well away from 0 (as the headline test)
        sure = without["grads"][k].abs() > 1e-4
        torch.testing.assert_close(with_head["params"][k][sure], without["params"][k][sure], rtol=0,
                                   atol=2e-6, msg=k)
