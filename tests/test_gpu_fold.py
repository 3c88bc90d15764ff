"""GPU parity of the Adam step folded into the two-layer backward's reduction
(include/ngnn.h ngnn_adam_fold, ABI 15): on one rank the graph slot's step
has no optimizer launch -- ngnn_sage2_bwd's k_bwd2_reduce updates every
parameter from the gradient it has just summed, with ngnn_adam_step's
arithmetic, and advances the same device step count.

Against the same slot with the fold disabled (the separate ngnn_adam_step
launch, itself checked against torch.optim.Adam by test_gpu_configs.py):
after three replays on different blocks the parameters, the Adam moments,
the step count and the last gradients agree -- bitwise for the parameters'
update arithmetic given identical gradients, so within the gradient bars
(the gradients' float atomics vary run to run).  An eager backward on the
slot's block never updates parameters.
"""
import pytest
import torch

import ngnn
from ngnn import fused

from gradbar import assert_wgrad

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _run(fold: bool):
    from ngnn.graphs import GraphedTrainStep, slot_size
    from ngnn.loader import sample_block, synthetic_graph
    from ngnn.optim import Adam
    torch.manual_seed(0)
    graph = synthetic_graph("ogbn-products", DEV, seed=5, scale=0.02)
    blocks = [sample_block(graph, graph.train_idx[512 * i:512 * (i + 1)], [15, 10], seed=20 + i)
              for i in range(4)]
    torch.manual_seed(0)
    model = ngnn.SAGE(100, 256, 47, 2, dropout=0.5).to(DEV).train()
    opt = Adam(model.parameters(), lr=1e-3, weight_decay=1e-4)
    n_cap, e_cap = slot_size(512, [15, 10])
    orig = fused.AdamFoldSpec.make
    if not fold:
        fused.AdamFoldSpec.make = staticmethod(lambda *a: None)
    try:
        step = GraphedTrainStep(model, opt, 512, n_cap, e_cap, 100, DEV)
        step.capture(blocks[3].x, blocks[3].edge_index, blocks[3].y)
    finally:
        fused.AdamFoldSpec.make = orig
    assert step.folded == fold and (step.g_opt is None) == fold
    losses = [float(step(b.x, b.edge_index, b.y)) for b in blocks[:3]]
    torch.cuda.synchronize()
    rec = dict(losses=losses,
               params={k: p.detach().clone() for k, p in model.named_parameters()},
               grads={k: p.grad.detach().clone() for k, p in model.named_parameters()},
               m={k: opt.state[p]["exp_avg"].clone() for k, p in model.named_parameters()},
               v={k: opt.state[p]["exp_avg_sq"].clone() for k, p in model.named_parameters()},
               step=float(opt.state[next(model.parameters())]["step"]))
    # eager on the slot's block: a backward alone leaves the parameters as they are
    before = {k: p.detach().clone() for k, p in model.named_parameters()}
    opt.zero_grad(set_to_none=False)
    from ngnn.losses import seed_cross_entropy
    seed_cross_entropy(model(step.x, step.ei), step.y, step.B).backward()
    torch.cuda.synchronize()
    for k, p in model.named_parameters():
        assert torch.equal(p.detach(), before[k]), f"an eager backward moved {k}"
    return rec


def test_adam_fold_matches_the_optimizer_launch():
    a, b = _run(True), _run(False)
    assert a["step"] == b["step"] == 3.0
    for x, y in zip(a["losses"], b["losses"]):
        assert abs(x - y) <= 1e-5 * max(1.0, abs(y))
    for k in b["params"]:
        assert_wgrad(a["grads"][k], b["grads"][k], msg=k)
        assert_wgrad(a["m"][k], b["m"][k], msg=k)
        torch.testing.assert_close(a["v"][k], b["v"][k], rtol=1e-3, atol=1e-12, msg=k)
        # the update is lr m / (sqrt(v) + eps): compared where |m| is away from 0
        sure = b["m"][k].abs() > 1e-5
        torch.testing.assert_close(a["params"][k][sure], b["params"][k][sure], rtol=0, atol=5e-6, msg=k)
