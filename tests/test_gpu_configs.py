"""Parity at the exact BASELINE.json configurations, through what bench.py
times.

Each test runs the benched step -- ngnn.graphs.GraphedTrainStep: slot load,
one captured forward (fused layer kernels, hash dropout), seed-row cross
entropy, bounded backward, Adam -- in TRAIN mode at the config's real model
dimensions and fanout on a full-size synthetic graph (datasets are not
downloadable; the graphs have the published node / edge / feature / class
counts), and checks it against the CPU oracle (oracle/pyg_ref.py: the PyG
2.5.1 op sequence) with the replay's dropout masks rebuilt on the host:

* the headline: ogbn-products SAGE(100,256,47) [15,10] bs 1024 (zero-copy
  slot): logits, loss, every gradient, post-step parameters;
* config #2, ogbn-arxiv SAGE(128,256,40) [15,10] bs 1024: the same;
* config #3, ogbn-products SAGE(100,256,256,47) bf16 [20,15,10] bs 1024:
  seed-row logits, loss and every gradient through the seeds' receptive
  field, a row sample's logits, post-step parameters -- bf16 against the
  fp32 oracle at the SURVEY 8(c) bf16 tolerance 2e-2;
* config #5, Amazon-Computers SAGE(767,512,10) max [10,5], 300 seeds
  (K % 4 != 0: the slot copies the rows): logits, then the backward layer
  by layer on the step's own per-layer tensors (near-tied maxima);
* config #1's widths, a CitationFull-Cora SAGE(8710,512,70) [10,5] bs 512.

Tolerances as tests/test_gpu_fused.py: outputs 1e-5, input gradients
rtol 1e-4 / atol 1e-5, weight gradients max|g - g_ref| <= 1e-5 max|g_ref|
(tests/gradbar.py); bf16 2e-2.
"""
import pytest
import torch
import torch.nn.functional as F

import ngnn
from oracle import pyg_ref

from test_gpu_fused import GRAD, OUT, _MaskedGCN, _MaskedSAGE, dropout_keep, dropout_scale
from gradbar import assert_wgrad

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _graph(name, seed=0, **kw):
    from ngnn.loader import synthetic_graph
    return synthetic_graph(name, DEV, seed=seed, **kw)


def _hooked_capture(step, x, ei, y):
    """step.capture with fused._debug_acts on: the captured forward's hidden
    activations (rewritten by every replay) kept as step._test_acts."""
    from ngnn import fused
    fused._debug_acts = []
    try:
        step.capture(x, ei, y)
        step._test_acts = fused._debug_acts[-1]
    finally:
        fused._debug_acts = None


def _gpu_hidden(step):
    """(the last replay's hidden activations on the host, the rows it wrote:
    the slot's R')."""
    return [a.cpu() for a in step._test_acts], int(step.r_next.item()) & 0xFFFFFFFF


def _eager_vs_oracle(b, mine, hidden, train, aggr, seed=99, out_tol=OUT, check_dx=False):
    """One eager forward + seed-row cross entropy + backward of `mine` on
    block `b` against the oracle with the same dropout masks."""
    N = b.num_nodes
    L = len(mine.convs)
    if train:
        torch.manual_seed(seed)
        s = int(torch.randint(0, 2**62, (1,)).item())
        torch.manual_seed(seed)
    mine.train(train)
    x = b.x.clone().requires_grad_(check_dx)
    out = mine(x, b.edge_index)
    F.cross_entropy(out[:b.batch_size], b.y[:b.batch_size]).backward()
    in_dim = b.x.size(1)
    C = mine.convs[-1].lin_r.weight.shape[0]
    if train:
        masks = [dropout_keep(s + 7919 * i, N, hidden, mine.dropout).float() for i in range(L - 1)]
        ref = _MaskedSAGE(in_dim, hidden, C, L, dropout=mine.dropout, aggr=aggr, masks=masks)
    else:
        ref = pyg_ref.SAGE(in_dim, hidden, C, L, dropout=mine.dropout, aggr=aggr).eval()
    ref.load_state_dict({k: v.float().cpu() for k, v in mine.state_dict().items()})
    xr = b.x.float().cpu().clone().requires_grad_(check_dx)
    out_r = ref(xr, b.edge_index.cpu())
    F.cross_entropy(out_r[:b.batch_size], b.y[:b.batch_size].cpu()).backward()
    torch.testing.assert_close(out.detach().float().cpu(), out_r.detach(), **out_tol)
    if check_dx:
        torch.testing.assert_close(x.grad.cpu(), xr.grad, **GRAD)
    for (k, p), (_, q) in zip(mine.named_parameters(), ref.named_parameters()):
        assert_wgrad(p.grad.cpu(), q.grad, msg=k)


@pytest.mark.timeout(300)
def test_headline_graph_step_full_products_block():
    """The benched step (bench.py: GraphedTrainStep over a zero-copy slot)
    on a full ogbn-products [15,10] bs 1024 block, train mode (dropout 0.5,
    hash masks rebuilt on the host from the slot's device seed)."""
    from ngnn.graphs import GraphedTrainStep, slot_size
    from ngnn.loader import sample_block
    from ngnn.optim import Adam
    g = _graph("ogbn-products")
    b = sample_block(g, g.train_idx[:1024], [15, 10], seed=7)
    b2 = sample_block(g, g.train_idx[1024:2048], [15, 10], seed=8)
    N = b.num_nodes
    assert b.edge_index.shape[1] > 150_000 and N > 140_000  # a full-size block
    torch.manual_seed(0)
    mine = ngnn.SAGE(100, 256, 47, 2, dropout=0.5).to(DEV).train()
    init = {k: v.detach().cpu().clone() for k, v in mine.state_dict().items()}
    opt = Adam(mine.parameters(), lr=1e-3)
    n_cap, e_cap = slot_size(1024, [15, 10])
    step = GraphedTrainStep(mine, opt, 1024, n_cap, e_cap, 100, DEV)
    _hooked_capture(step, b2.x, b2.edge_index, b2.y)  # warm-up on another block; state restored
    loss = step(b.x, b.edge_index, b.y)
    torch.cuda.synchronize()
    assert step.zero_copy
    out = step.out[:N].cpu()
    grads = {k: p.grad.detach().cpu().clone() for k, p in mine.named_parameters()}
    seed_state = int(step.seed_state.item()) & (2**64 - 1)
    masks = [dropout_keep((7919 * i) ^ seed_state, N, 256, 0.5).float() for i in range(1)]
    hid, rn = _gpu_hidden(step)
    ref = _MaskedSAGE(100, 256, 47, 2, dropout=0.5, masks=masks, gpu_hidden=hid, kink_rows=rn)
    ref.load_state_dict(init)
    out_r = ref(b.x.cpu(), b.edge_index.cpu())
    loss_r = F.cross_entropy(out_r[:1024], b.y[:1024].cpu())
    loss_r.backward()
    torch.testing.assert_close(out, out_r.detach(), **OUT)
    assert abs(float(loss) - float(loss_r)) < 1e-5
    for k, q in ref.named_parameters():
        assert_wgrad(grads[k], q.grad, msg=k)
    # post-step parameters: torch's Adam on the oracle's gradients.  At step 1
    # the update is lr * g / (|g| + eps): compare where |g| is well away from 0
    # (elsewhere a 1e-7 gradient difference may flip the sign of a 1e-3 step)
    o_ref = torch.optim.Adam(ref.parameters(), lr=1e-3)
    o_ref.step()
    for k, q in ref.named_parameters():
        p = dict(mine.named_parameters())[k].detach().cpu()
        sure = q.grad.abs() > 1e-4
        torch.testing.assert_close(p[sure], q.detach()[sure], rtol=0, atol=2e-6, msg=k)
        assert (p - init[k]).abs().max() <= 1e-3 + 1e-6, k
    _check_step1_state(step, mine, ref)
    b3 = sample_block(g, g.train_idx[2048:3072], [15, 10], seed=9)
    _check_second_step(step, mine, b3, 100, 256, 47, 2, 1024)


@pytest.mark.timeout(300)
def test_headline_graph_step_fused_row_gather_vs_oracle():
    """the headline step with the fused x[n_id] gather
    (NeighborLoader(gather_features=False): the batch hands the resident
    feature table + n_id; layer 0's kernels and weight gradient read table
    rows n_id[r]) against the oracle on the MATERIALIZED rows -- logits of
    every row, loss, every gradient, post-step parameters."""
    from ngnn.graphs import GraphedTrainStep, slot_size
    from ngnn.loader import IndexedRows, sample_block
    from ngnn.optim import Adam
    g = _graph("ogbn-products")
    b = sample_block(g, g.train_idx[:1024], [15, 10], seed=17)
    b2 = sample_block(g, g.train_idx[1024:2048], [15, 10], seed=18)
    N = b.num_nodes
    torch.manual_seed(3)
    mine = ngnn.SAGE(100, 256, 47, 2, dropout=0.5).to(DEV).train()
    init = {k: v.detach().cpu().clone() for k, v in mine.state_dict().items()}
    opt = Adam(mine.parameters(), lr=1e-3)
    n_cap, e_cap = slot_size(1024, [15, 10])
    step = GraphedTrainStep(mine, opt, 1024, n_cap, e_cap, 100, DEV)
    _hooked_capture(step, IndexedRows(g.x, b2.n_id), b2.edge_index, b2.y)
    assert step.zero_copy and step.x_rows == g.num_nodes
    loss = step(IndexedRows(g.x, b.n_id), b.edge_index, b.y)
    torch.cuda.synchronize()
    out = step.out[:N].cpu()
    grads = {k: p.grad.detach().cpu().clone() for k, p in mine.named_parameters()}
    seed_state = int(step.seed_state.item()) & (2**64 - 1)
    hid, rn = _gpu_hidden(step)
    ref = _MaskedSAGE(100, 256, 47, 2, dropout=0.5, gpu_hidden=hid, kink_rows=rn,
                      masks=[dropout_keep(seed_state, N, 256, 0.5).float()])
    ref.load_state_dict(init)
    xm = g.x[b.n_id].cpu()  # the materialized rows
    assert torch.equal(xm, b.x.cpu())
    out_r = ref(xm, b.edge_index.cpu())
    loss_r = F.cross_entropy(out_r[:1024], b.y[:1024].cpu())
    loss_r.backward()
    torch.testing.assert_close(out, out_r.detach(), **OUT)
    assert abs(float(loss) - float(loss_r)) < 1e-5
    for k, q in ref.named_parameters():
        assert_wgrad(grads[k], q.grad, msg=k)
    o_ref = torch.optim.Adam(ref.parameters(), lr=1e-3)
    o_ref.step()
    for k, q in ref.named_parameters():
        p = dict(mine.named_parameters())[k].detach().cpu()
        sure = q.grad.abs() > 1e-4
        torch.testing.assert_close(p[sure], q.detach()[sure], rtol=0, atol=2e-6, msg=k)
    _check_step1_state(step, mine, ref)


def _graph_step(model, b, warm, fanout, bs, in_dim, lr=1e-3):
    """The benched step: GraphedTrainStep (slot load + one captured forward,
    seed-row cross entropy, bounded backward, Adam) on block b after a
    capture (warm-up state restored) on block `warm`.  Returns the step, its
    loss and the slot's dropout seed of that replay."""
    from ngnn.graphs import GraphedTrainStep, slot_size
    from ngnn.optim import Adam
    opt = Adam(model.parameters(), lr=lr)
    n_cap, e_cap = slot_size(bs, fanout)
    step = GraphedTrainStep(model, opt, bs, n_cap, e_cap, in_dim, DEV)
    _hooked_capture(step, warm.x, warm.edge_index, warm.y)
    loss = step(b.x, b.edge_index, b.y)
    torch.cuda.synchronize()
    return step, loss, int(step.seed_state.item()) & (2**64 - 1)


def _slot_masks(seed_state, N, hidden, p, L):
    """The dropout keep masks of a graph replay (layer i keyed by the slot
    seed: (7919 i) ^ seed_state)."""
    return [dropout_keep((7919 * i) ^ seed_state, N, hidden, p).float() for i in range(L - 1)]


def _check_second_step(step, mine, b2, in_dim, hidden, C, L, bs, lr=1e-3, aggr="mean", gcn=False):
    """Adam step 2, where the update depends on |g| (at step
    1 it is ~lr * sign(g)).  The step-1 Adam state the GPU kept (exp_avg =
    0.1 g1, exp_avg_sq = 0.001 g1^2) is checked against the oracle's step-1
    gradients (caller: q.grad) by the gradient bar; then a second replay on
    block b2, and the oracle -- started from the GPU's step-1 parameters and
    Adam state, so both sides see identical inputs -- takes the same step:
    its gradients at the bar, the loss at 1e-5, the parameters after torch's
    Adam step 2 at 2e-6 where |g1|, |g2| >= 1e-2 of their tensor's max."""
    named = dict(mine.named_parameters())
    p1 = {k: p.detach().cpu().clone() for k, p in named.items()}
    st1 = {k: (step.opt.state[p]["exp_avg"].detach().cpu().clone(),
               step.opt.state[p]["exp_avg_sq"].detach().cpu().clone()) for k, p in named.items()}
    loss2 = step(b2.x, b2.edge_index, b2.y)
    torch.cuda.synchronize()
    seed2 = int(step.seed_state.item()) & (2**64 - 1)
    grads2 = {k: p.grad.detach().cpu().clone() for k, p in named.items()}
    N2 = b2.num_nodes
    hid, rn = _gpu_hidden(step)
    masks2 = _slot_masks(seed2, N2, hidden, 0.5, L)
    if gcn:
        ref2 = _MaskedGCN(in_dim, hidden, C, L, dropout=0.5, masks=masks2, gpu_hidden=hid, kink_rows=rn)
    else:
        ref2 = _MaskedSAGE(in_dim, hidden, C, L, dropout=0.5, aggr=aggr, masks=masks2, gpu_hidden=hid,
                           kink_rows=rn)
    ref2.load_state_dict(p1)
    out2 = ref2(b2.x.cpu(), b2.edge_index.cpu())
    loss_r2 = F.cross_entropy(out2[:bs], b2.y[:bs].cpu())
    loss_r2.backward()
    assert abs(float(loss2) - float(loss_r2)) < 1e-5 * (max(1.0, abs(float(loss_r2))) if gcn else 1.0)
    for k, q in ref2.named_parameters():
        assert_wgrad(grads2[k], q.grad, msg=f"step2:{k}")
    o2 = torch.optim.Adam(ref2.parameters(), lr=lr)
    for k, q in ref2.named_parameters():
        o2.state[q] = dict(step=torch.tensor(1.0), exp_avg=st1[k][0].clone(), exp_avg_sq=st1[k][1].clone())
    o2.step()
    for k, q in ref2.named_parameters():
        p = named[k].detach().cpu()
        g1 = st1[k][0] / 0.1
        sure = (g1.abs() >= 1e-2 * g1.abs().max()) & (q.grad.abs() >= 1e-2 * q.grad.abs().max())
        assert int(sure.sum()) > 0, k
        torch.testing.assert_close(p[sure], q.detach()[sure], rtol=0, atol=2e-6, msg=f"step2:{k}")


def _check_step1_state(step, mine, ref):
    """The step-1 Adam moments the GPU kept are (1 - beta1) g and (1 - beta2)
    g^2 of ITS gradients (the factors as fp32 computes them: 1 - 0.999f is
    0.0010000467): against the oracle's gradients at the bar."""
    one = torch.tensor(1.0, dtype=torch.float32)
    c1 = float(one - torch.tensor(0.9, dtype=torch.float32))
    c2 = float(one - torch.tensor(0.999, dtype=torch.float32))
    for k, q in ref.named_parameters():
        p = dict(mine.named_parameters())[k]
        assert_wgrad(step.opt.state[p]["exp_avg"].cpu().double() / c1, q.grad, msg=f"exp_avg:{k}")
        v = step.opt.state[p]["exp_avg_sq"].cpu().double() / c2
        assert_wgrad(v.sqrt(), q.grad.double().abs(), msg=f"exp_avg_sq:{k}")


def _check_adam_step(mine, ref, init, lr=1e-3, bf16=False):
    """Post-step parameters against torch's Adam on the oracle's gradients.
    At step 1 the update is lr * g / (|g| + eps): compared where |g| is well
    away from 0 (elsewhere a tiny gradient difference may flip a 1e-3 step);
    bf16 parameters within one bf16 rounding of the oracle's update."""
    o_ref = torch.optim.Adam(ref.parameters(), lr=lr)
    o_ref.step()
    for k, q in ref.named_parameters():
        p = dict(mine.named_parameters())[k].detach().float().cpu()
        sure = q.grad.abs() > (1e-3 if bf16 else 1e-4) * max(1.0, float(q.grad.abs().max()))
        want = q.detach()
        if bf16:
            want = want.to(torch.bfloat16).float()
            tol = want.abs() * 2.0**-7 + 1e-6
            assert ((p - want).abs() <= tol)[sure].all(), k
        else:
            torch.testing.assert_close(p[sure], want[sure], rtol=0, atol=2e-6, msg=k)
        # |step| <= lr (plus, for bf16, the rounding of the new value)
        bound = lr + 1e-6 + (torch.maximum(init[k].abs(), p.abs()) * 2.0**-7 if bf16 else 0.0)
        assert ((p - init[k]).abs() <= bound).all(), k


@pytest.mark.timeout(300)
def test_gcn_headline_graph_step_two_layer_kernels():
    """`bench.py --module gcn`: SimpleGCN(100,256,47) (convolution.py:7-35,
    GCNConv(normalize=False)) on a full ogbn-products [15,10] bs 1024 block
    through the benched graph step -- now the two-layer kernels with W_r = 0
    (fused.sage2_params), the loss head and the Adam fold: logits of every
    row, loss, every gradient, the step-1 Adam state and Adam step 2."""
    from ngnn import fused
    from ngnn.loader import sample_block
    g = _graph("ogbn-products")
    b = sample_block(g, g.train_idx[:1024], [15, 10], seed=27)
    warm = sample_block(g, g.train_idx[1024:2048], [15, 10], seed=28)
    torch.manual_seed(5)
    mine = ngnn.SimpleGCN(100, 256, 47, 2, dropout=0.5).to(DEV).train()
    init = {k: v.detach().cpu().clone() for k, v in mine.state_dict().items()}
    calls = []
    orig = fused.sage2_forward

    def spy(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    fused.sage2_forward = spy
    try:
        step, loss, seed_state = _graph_step(mine, b, warm, [15, 10], 1024, 100)
    finally:
        fused.sage2_forward = orig
    assert calls, "the GCN stack did not take ngnn_sage2_fwd"
    assert step.zero_copy and step.folded and step._head is not None
    N = b.num_nodes
    out = step.out[:N].cpu()
    grads = {k: p.grad.detach().cpu().clone() for k, p in mine.named_parameters()}
    hid, rn = _gpu_hidden(step)
    ref = _MaskedGCN(100, 256, 47, 2, dropout=0.5, masks=_slot_masks(seed_state, N, 256, 0.5, 2),
                     gpu_hidden=hid, kink_rows=rn)
    ref.load_state_dict(init)
    out_r = ref(b.x.cpu(), b.edge_index.cpu())
    loss_r = F.cross_entropy(out_r[:1024], b.y[:1024].cpu())
    loss_r.backward()
    # sum aggregation: outputs grow with degree x width (test_gcn_stack_fwd_bwd_matches_oracle)
    scale = max(1.0, float(out_r.detach().abs().max()))
    torch.testing.assert_close(out, out_r.detach(), rtol=OUT["rtol"], atol=OUT["atol"] * scale)
    assert abs(float(loss) - float(loss_r)) < 1e-5 * max(1.0, abs(float(loss_r)))
    for k, q in ref.named_parameters():
        assert_wgrad(grads[k], q.grad, msg=k)
    _check_step1_state(step, mine, ref)
    _check_second_step(step, mine, sample_block(g, g.train_idx[2048:3072], [15, 10], seed=29),
                       100, 256, 47, 2, 1024, gcn=True)


@pytest.mark.timeout(300)
def test_config_arxiv_graph_step():
    """BASELINE config #2: ogbn-arxiv SAGE(128,256,40), [15,10] bs 1024, fp32,
    through the benched graph step in train mode (dropout 0.5): logits of
    every row, loss, every gradient and the post-step parameters."""
    from ngnn.loader import sample_block
    g = _graph("ogbn-arxiv")
    b = sample_block(g, g.train_idx[:1024], [15, 10], seed=3)
    warm = sample_block(g, g.train_idx[1024:2048], [15, 10], seed=4)
    torch.manual_seed(1)
    mine = ngnn.SAGE(128, 256, 40, 2, dropout=0.5).to(DEV).train()
    init = {k: v.detach().cpu().clone() for k, v in mine.state_dict().items()}
    step, loss, seed_state = _graph_step(mine, b, warm, [15, 10], 1024, 128)
    assert step.zero_copy
    N = b.num_nodes
    out = step.out[:N].cpu()
    grads = {k: p.grad.detach().cpu().clone() for k, p in mine.named_parameters()}
    hid, rn = _gpu_hidden(step)
    ref = _MaskedSAGE(128, 256, 40, 2, dropout=0.5, masks=_slot_masks(seed_state, N, 256, 0.5, 2),
                      gpu_hidden=hid, kink_rows=rn)
    ref.load_state_dict(init)
    out_r = ref(b.x.cpu(), b.edge_index.cpu())
    loss_r = F.cross_entropy(out_r[:1024], b.y[:1024].cpu())
    loss_r.backward()
    torch.testing.assert_close(out, out_r.detach(), **OUT)
    assert abs(float(loss) - float(loss_r)) < 1e-5
    for k, q in ref.named_parameters():
        assert_wgrad(grads[k], q.grad, msg=k)
    _check_adam_step(mine, ref, init)
    _check_step1_state(step, mine, ref)
    _check_second_step(step, mine, sample_block(g, g.train_idx[2048:3072], [15, 10], seed=5),
                       128, 256, 40, 2, 1024)


@pytest.mark.timeout(300)
def test_config_computers_max_graph_step():
    """BASELINE config #5: Amazon-Computers SAGE(767,512,10) max, [10,5], the
    config's full batch of 300 seeds, through the benched graph step in
    train mode (K = 767: not a multiple of 4, so the slot copies the rows).

    Logits of every row at 1e-5.  The max gradient goes to the argmax
    neighbour, and fp32 rounding differences between the GPU's and the CPU's
    layer-0 outputs (~1e-6) flip near-tied maxima, so the backward is pinned
    LAYER BY LAYER on identical inputs: the captured step's own per-layer
    tensors (the debug hook's clones, recorded into the graph and rewritten
    by every replay) feed the oracle's layer backward.  Post-step parameters
    against torch's Adam on the GPU gradients' oracle counterparts."""
    from ngnn import fused
    from ngnn.loader import sample_block
    g = _graph("computers")
    b = sample_block(g, g.train_idx, [10, 5], seed=5)
    warm = sample_block(g, g.train_idx, [10, 5], seed=6)
    assert b.batch_size == 300
    torch.manual_seed(2)
    mine = ngnn.SAGE(767, 512, 10, 2, dropout=0.5, aggr="max").to(DEV).train()
    init = {k: v.detach().cpu().clone() for k, v in mine.state_dict().items()}
    fused._debug_grads = []
    try:
        step, loss, seed_state = _graph_step(mine, b, warm, [10, 5], 300, 767)
        captured = fused._debug_grads[-2:]  # the captured backward's entries (layers 1, 0)
        dbg = {i: (dy.cpu(), hin.cpu()) for i, dy, _, hin in captured}
    finally:
        fused._debug_grads = None
    assert sorted(dbg) == [0, 1]
    N = b.num_nodes
    out = step.out[:N].cpu()
    grads = {k: p.grad.detach().cpu().clone() for k, p in mine.named_parameters()}
    mask = _slot_masks(seed_state, N, 512, 0.5, 2)[0]
    ref = _MaskedSAGE(767, 512, 10, 2, dropout=0.5, aggr="max", masks=[mask])
    ref.load_state_dict(init)
    x, ei, y = b.x.cpu(), b.edge_index.cpu(), b.y[:300].cpu()
    with torch.no_grad():
        out_r = ref(x, ei)
    torch.testing.assert_close(out, out_r, **OUT)
    assert abs(float(loss) - float(F.cross_entropy(out_r[:300], y))) < 1e-5
    # the layer-1 input the step saw is the oracle's layer-0 output (1e-5)
    with torch.no_grad():
        h0 = ref.convs[0](x, ei).relu() * mask * dropout_scale(0.5)
    torch.testing.assert_close(dbg[1][1][:N], h0, **OUT)
    # layer 1 on the GPU's layer-1 input
    h1 = dbg[1][1][:N].clone().requires_grad_(True)
    F.cross_entropy(ref.convs[1](h1, ei)[:300], y).backward()
    src, dst = ei
    rn = max(300, int(src[dst < 300].max()) + 1)
    assert not h1.grad[rn:].any()
    torch.testing.assert_close(dbg[0][0][:rn], h1.grad[:rn], **GRAD)
    for n, q in ref.convs[1].named_parameters():
        assert_wgrad(grads[f"convs.1.{n}"], q.grad, msg=n)
    # layer 0 (relu + dropout) under the GPU's output gradient
    h0 = ref.convs[0](x, ei).relu() * mask * dropout_scale(0.5)
    h0.backward(torch.cat([dbg[0][0][:rn], torch.zeros(N - rn, 512)]))
    for n, q in ref.convs[0].named_parameters():
        assert_wgrad(grads[f"convs.0.{n}"], q.grad, msg=n)
    _check_adam_step(mine, ref, init)


@pytest.mark.timeout(300)
def test_config_cora_width_graph_step():
    """BASELINE config #1's layer widths: CitationFull-Cora SAGE(8710,512,70)
    (config_cora.yml fanout [10,5], bs 512) on a Cora-sized synthetic graph,
    through the graph step in train mode (K = 8,710: the W_r image exceeds
    the LDS, the 64-row kernel's path)."""
    from ngnn.loader import sample_block
    g = _graph("cora")
    b = sample_block(g, g.train_idx[:512], [10, 5], seed=9)
    warm = sample_block(g, g.train_idx[512:1024], [10, 5], seed=10)
    torch.manual_seed(3)
    mine = ngnn.SAGE(8710, 512, 70, 2, dropout=0.5).to(DEV).train()
    init = {k: v.detach().cpu().clone() for k, v in mine.state_dict().items()}
    step, loss, seed_state = _graph_step(mine, b, warm, [10, 5], 512, 8710)
    N = b.num_nodes
    out = step.out[:N].cpu()
    grads = {k: p.grad.detach().cpu().clone() for k, p in mine.named_parameters()}
    hid, rn = _gpu_hidden(step)
    ref = _MaskedSAGE(8710, 512, 70, 2, dropout=0.5, masks=_slot_masks(seed_state, N, 512, 0.5, 2),
                      gpu_hidden=hid, kink_rows=rn)
    ref.load_state_dict(init)
    out_r = ref(b.x.cpu(), b.edge_index.cpu())
    loss_r = F.cross_entropy(out_r[:512], b.y[:512].cpu())
    loss_r.backward()
    torch.testing.assert_close(out, out_r.detach(), **OUT)
    assert abs(float(loss) - float(loss_r)) < 1e-5
    for k, q in ref.named_parameters():
        assert_wgrad(grads[k], q.grad, msg=k)
    _check_adam_step(mine, ref, init)
    _check_step1_state(step, mine, ref)
    _check_second_step(step, mine, sample_block(g, g.train_idx[:512], [10, 5], seed=11),
                       8710, 512, 70, 2, 512)


def _receptive_rows(ei, rows, hops):
    """Row sets needed layer by layer: S_L = rows, S_{l-1} = S_l + sources of
    the edges into S_l."""
    src, dst = ei
    sets = [rows]
    for _ in range(hops):
        cur = sets[-1]
        m = torch.zeros(int(max(src.max(), dst.max())) + 1, dtype=torch.bool)
        m[cur] = True
        sets.append(torch.unique(torch.cat([cur, src[m[dst]]])))
    return sets[::-1]


def _oracle_rows(ref, x, ei, rows, masks=None, scale=1.0, act_dtype=None):
    """The oracle's outputs for `rows` only, computed through their receptive
    field (layer l over the rows layer l+1 needs, with every edge into them):
    the same values as the full-block forward on those rows.  masks: the
    hidden layers' dropout keep masks over the whole block (row-indexed).
    act_dtype: each hidden layer's output stored in that dtype (a bf16
    model's activations, as the reference's bf16 layers hand them on); the
    rounding is straight-through for the gradient (kept fp32, as ours)."""
    L = len(ref.convs)
    sets = _receptive_rows(ei, rows, L)
    src, dst = ei
    n = int(ei.max()) + 1
    h, have = x[sets[0]], sets[0]
    for i, conv in enumerate(ref.convs):
        need = sets[i + 1]
        pos = torch.full((n,), -1, dtype=torch.long)
        pos[have] = torch.arange(have.numel())
        keep = torch.zeros(n, dtype=torch.bool)
        keep[need] = True
        e = keep[dst]  # every edge into a needed row (its source is in `have`)
        h = conv(h, torch.stack([pos[src[e]], pos[dst[e]]]))[pos[need]]
        if i != L - 1:
            h = h.relu()
            if masks is not None:
                h = h * masks[i][need] * scale
            if act_dtype is not None:
                h = h + (h.to(act_dtype).float() - h).detach()
        have = need
    return h


@pytest.mark.timeout(400)
def test_config_products_3layer_bf16_graph_step():
    """BASELINE config #3: ogbn-products SAGE(100,256,256,47) in bf16,
    [20,15,10] bs 1024, through the benched graph step in TRAIN mode
    (dropout 0.5, hash masks from the slot seed).  Against the fp32 oracle
    with the bf16 model's storage points (features, parameters, the hidden
    layers' activations -- rounded to bf16 as the reference's bf16 layers
    store them --, logits, gradients) at the SURVEY 8(c) bf16 tolerance 2e-2:

    * logits of the seed rows and of a row sample, through their receptive
      field (the oracle over the whole 1.5 M-row block is not needed: the
      loss reads the seed rows, whose receptive field IS the block's
      training-relevant part);
    * the loss and every parameter gradient (seed-row loss back-propagated
      through that receptive field: exactly the full block's gradients),
      elementwise at 2e-2 of the tensor's largest magnitude;
    * the post-step parameters within one bf16 rounding of torch's Adam."""
    from ngnn.loader import sample_block
    g = _graph("ogbn-products")
    g.x = g.x.to(torch.bfloat16)
    b = sample_block(g, g.train_idx[:1024], [20, 15, 10], seed=11)
    warm = sample_block(g, g.train_idx[1024:2048], [20, 15, 10], seed=12)
    torch.manual_seed(4)
    mine = ngnn.SAGE(100, 256, 47, 3, dropout=0.5).to(DEV).to(torch.bfloat16).train()
    init = {k: v.detach().float().cpu().clone() for k, v in mine.state_dict().items()}
    step, loss, seed_state = _graph_step(mine, b, warm, [20, 15, 10], 1024, 100)
    N = b.num_nodes
    # the slot's loss reads the seed rows: the bf16 logits hold those rows,
    # every row's logits stay in fp32 (step.out_f32; round 6)
    assert step.out_f32 is not None
    out = torch.cat([step.out[:1024].float(), step.out_f32[1024:N].to(torch.bfloat16).float()]).cpu()
    assert torch.isfinite(out).all()
    grads = {k: p.grad.detach().float().cpu().clone() for k, p in mine.named_parameters()}
    masks = _slot_masks(seed_state, N, 256, 0.5, 3)
    ref = pyg_ref.SAGE(100, 256, 47, 3, dropout=0.5)
    ref.load_state_dict(init)
    x, ei = b.x.float().cpu(), b.edge_index.cpu()
    seeds = torch.arange(1024)
    out_r = _oracle_rows(ref, x, ei, seeds, masks, dropout_scale(0.5), act_dtype=torch.bfloat16)
    loss_r = F.cross_entropy(out_r, b.y[:1024].cpu())
    loss_r.backward()
    BF = dict(rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(out[:1024], out_r.detach(), **BF)
    assert abs(float(loss) - float(loss_r)) < 2e-2 * max(1.0, abs(float(loss_r)))
    for k, q in ref.named_parameters():
        d = (grads[k] - q.grad).abs()
        torch.testing.assert_close(
            grads[k], q.grad, rtol=2e-2, atol=2e-2 * float(q.grad.abs().max()),
            msg=f"{k}: max |diff| {float(d.max()):.3g} at {int(d.argmax())}, |ref| max "
                f"{float(q.grad.abs().max()):.3g}, mine there {float(grads[k].flatten()[d.argmax()]):.3g} "
                f"ref there {float(q.grad.flatten()[d.argmax()]):.3g}")
    gen = torch.Generator().manual_seed(0)
    rows = torch.unique(torch.randint(1024, N, (3000,), generator=gen))
    with torch.no_grad():
        want = _oracle_rows(ref, x, ei, rows, masks, dropout_scale(0.5), act_dtype=torch.bfloat16)
    torch.testing.assert_close(out[rows], want, **BF)
    _check_adam_step(mine, ref, init, bf16=True)


def test_3layer_h256_backward_gemm_scatter_path():
    """SAGE(100,256,256,47), train mode, input gradient wanted: the 256 x 256
    and 100 -> 256 layers' input gradients run the dgrad GEMM + scatter
    (weights too large for the fused kernel's LDS); every gradient against
    the oracle."""
    from ngnn.fused import _dgrad_fused_ok
    from ngnn.loader import sample_block
    assert not _dgrad_fused_ok(256, 256) and not _dgrad_fused_ok(256, 100)
    g = _graph("ogbn-products", scale=0.01)
    b = sample_block(g, g.train_idx[:256], [8, 5, 3], seed=5)
    torch.manual_seed(7)
    mine = ngnn.SAGE(100, 256, 47, 3, dropout=0.5).to(DEV)
    _eager_vs_oracle(b, mine, 256, train=True, aggr="mean", check_dx=True)
