"""Parity at the exact BASELINE.json configurations.

Each test runs the product path at the config's real model dimensions and
fanout on a full-size synthetic graph (datasets are not downloadable; the
graphs have the published node / edge / feature / class counts) and checks it
against the CPU oracle (oracle/pyg_ref.py: the PyG 2.5.1 op sequence):

* the headline path itself -- GraphedTrainStep (zero-copy slot, captured
  forward + bounded backward + Adam, hash dropout) -- on a full
  ogbn-products [15,10] bs 1024 block: logits, every gradient and the
  post-step parameters;
* ogbn-arxiv SAGE(128,256,40) [15,10] bs 1024, train mode;
* Amazon-Computers SAGE(767,512,10) max [10,5], 300 seeds (K % 4 != 0);
* ogbn-products SAGE(100,256,256,47) bf16 [20,15,10] bs 1024 in the graph
  slot (slot rows x 256 fp32 > 2 GiB: the 64-row kernel and the slot copy),
  bf16 against the fp32 oracle at the SURVEY 8(c) bf16 tolerance, on the
  seed rows and a row sample through the oracle's receptive field;
* a CitationFull-Cora-width layer stack SAGE(8710,512,70).

Tolerances as tests/test_gpu_fused.py: outputs 1e-5, input gradients
rtol 1e-4 / atol 1e-5, weight gradients 1e-4; bf16 2e-2.
"""
import pytest
import torch
import torch.nn.functional as F

import ngnn
from oracle import pyg_ref

from test_gpu_fused import GRAD, OUT, WGRAD, _MaskedSAGE, dropout_keep, dropout_scale

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _graph(name, seed=0, **kw):
    from ngnn.loader import synthetic_graph
    return synthetic_graph(name, DEV, seed=seed, **kw)


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
        torch.testing.assert_close(p.grad.cpu(), q.grad, **WGRAD, msg=k)


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
    step.capture(b2.x, b2.edge_index, b2.y)  # warm-up on another block; state restored
    loss = step(b.x, b.edge_index, b.y)
    torch.cuda.synchronize()
    assert step.zero_copy
    out = step.out[:N].cpu()
    grads = {k: p.grad.detach().cpu().clone() for k, p in mine.named_parameters()}
    seed_state = int(step.seed_state.item()) & (2**64 - 1)
    masks = [dropout_keep((7919 * i) ^ seed_state, N, 256, 0.5).float() for i in range(1)]
    ref = _MaskedSAGE(100, 256, 47, 2, dropout=0.5, masks=masks)
    ref.load_state_dict(init)
    out_r = ref(b.x.cpu(), b.edge_index.cpu())
    loss_r = F.cross_entropy(out_r[:1024], b.y[:1024].cpu())
    loss_r.backward()
    torch.testing.assert_close(out, out_r.detach(), **OUT)
    assert abs(float(loss) - float(loss_r)) < 1e-5
    for k, q in ref.named_parameters():
        torch.testing.assert_close(grads[k], q.grad, **WGRAD, msg=k)
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


@pytest.mark.timeout(300)
def test_config_arxiv_15_10_bs1024():
    from ngnn.loader import sample_block
    g = _graph("ogbn-arxiv")
    b = sample_block(g, g.train_idx[:1024], [15, 10], seed=3)
    torch.manual_seed(1)
    mine = ngnn.SAGE(128, 256, 40, 2, dropout=0.5).to(DEV)
    _eager_vs_oracle(b, mine, 256, train=True, aggr="mean", check_dx=True)


@pytest.mark.timeout(300)
def test_config_computers_max_10_5():
    """K = 767 (not a multiple of 4), max aggregator, the config's full batch.

    Forward end to end at 1e-5.  The max gradient goes to the argmax
    neighbour, and fp32 rounding differences between the GPU's and the CPU's
    layer-0 outputs (~1e-6) flip near-tied maxima (~1e6 (row, feature) pairs
    here), so the backward is pinned LAYER BY LAYER on identical inputs: the
    oracle's layer-1 backward runs on the GPU's layer-1 input, the oracle's
    layer-0 backward on the GPU's layer-0 output gradient."""
    from ngnn import fused
    from ngnn.loader import sample_block
    g = _graph("computers")
    b = sample_block(g, g.train_idx, [10, 5], seed=5)
    assert b.batch_size == 300
    torch.manual_seed(2)
    mine = ngnn.SAGE(767, 512, 10, 2, dropout=0.5, aggr="max").to(DEV).train()
    torch.manual_seed(99)
    s = int(torch.randint(0, 2**62, (1,)).item())
    torch.manual_seed(99)
    fused._debug_grads = []
    try:
        out = mine(b.x, b.edge_index)
        F.cross_entropy(out[:300], b.y[:300]).backward()
        dbg = {i: (dy.cpu(), hin.cpu()) for i, dy, _, hin in fused._debug_grads}
    finally:
        fused._debug_grads = None
    N = b.num_nodes
    mask = dropout_keep(s, N, 512, 0.5).float()
    ref = _MaskedSAGE(767, 512, 10, 2, dropout=0.5, aggr="max", masks=[mask])
    ref.load_state_dict({k: v.cpu() for k, v in mine.state_dict().items()})
    x, ei, y = b.x.cpu(), b.edge_index.cpu(), b.y[:300].cpu()
    with torch.no_grad():
        torch.testing.assert_close(out.cpu(), ref(x, ei), **OUT)
    grads = {k: p.grad.cpu() for k, p in mine.named_parameters()}
    # layer 1 on the GPU's layer-1 input
    h1 = dbg[1][1].clone().requires_grad_(True)
    F.cross_entropy(ref.convs[1](h1, ei)[:300], y).backward()
    # d(layer-1 input): the bounded backward writes rows < R' = max(R, 1 + max
    # source of the edges into rows < R) only -- the oracle is zero past them
    src, dst = ei
    rn = max(300, int(src[dst < 300].max()) + 1)
    assert not h1.grad[rn:].any()
    torch.testing.assert_close(dbg[0][0][:rn], h1.grad[:rn], **GRAD)
    for n, q in ref.convs[1].named_parameters():
        torch.testing.assert_close(grads[f"convs.1.{n}"], q.grad, **WGRAD, msg=n)
    # layer 0 (relu + dropout) under the GPU's output gradient
    h0 = ref.convs[0](x, ei).relu() * mask * dropout_scale(0.5)
    h0.backward(torch.cat([dbg[0][0][:rn], torch.zeros(N - rn, 512)]))
    for n, q in ref.convs[0].named_parameters():
        torch.testing.assert_close(grads[f"convs.0.{n}"], q.grad, **WGRAD, msg=n)


@pytest.mark.timeout(300)
def test_config_cora_width_stack():
    """CitationFull-Cora widths: 8,710 features -> 512 -> 70 (config_cora.yml
    fanout [10,5], bs 512) on a Cora-sized synthetic graph."""
    from ngnn.loader import sample_block
    g = _graph("cora")
    b = sample_block(g, g.train_idx[:512], [10, 5], seed=9)
    torch.manual_seed(3)
    mine = ngnn.SAGE(8710, 512, 70, 2, dropout=0.5).to(DEV)
    _eager_vs_oracle(b, mine, 512, train=True, aggr="mean")


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


def _oracle_rows(ref, x, ei, rows):
    """The oracle's outputs for `rows` only, computed through their receptive
    field (layer l over the rows layer l+1 needs, with every edge into them):
    the same values as the full-block forward on those rows."""
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
        have = need
    return h


@pytest.mark.timeout(400)
def test_config_products_3layer_bf16_graph_slot():
    """ogbn-products SAGE(100,256,256,47) in bf16, [20,15,10] bs 1024, through
    the graph step (eval-mode forward of the captured model on the slot): the
    slot's rows x 256 fp32 exceed the row-tile kernel's 2 GiB buffer range,
    so this is the large-block path.  bf16 against the fp32 oracle (2e-2),
    seed rows and a row sample, through their receptive field."""
    from ngnn.graphs import GraphedTrainStep, slot_size
    from ngnn.loader import sample_block
    from ngnn.optim import Adam
    g = _graph("ogbn-products")
    g.x = g.x.to(torch.bfloat16)
    b = sample_block(g, g.train_idx[:1024], [20, 15, 10], seed=11)
    torch.manual_seed(4)
    mine = ngnn.SAGE(100, 256, 47, 3, dropout=0.0).to(DEV).to(torch.bfloat16).train()
    init = {k: v.detach().float().cpu().clone() for k, v in mine.state_dict().items()}
    opt = Adam(mine.parameters(), lr=1e-3)
    n_cap, e_cap = slot_size(1024, [20, 15, 10])
    step = GraphedTrainStep(mine, opt, 1024, n_cap, e_cap, 100, DEV)
    step.capture(b.x, b.edge_index, b.y)
    step(b.x, b.edge_index, b.y)
    torch.cuda.synchronize()
    N = b.num_nodes
    out = step.out[:N].float().cpu()
    ref = pyg_ref.SAGE(100, 256, 47, 3, dropout=0.0).eval()
    ref.load_state_dict(init)
    gen = torch.Generator().manual_seed(0)
    rows = torch.unique(torch.cat([torch.arange(1024), torch.randint(1024, N, (3000,), generator=gen)]))
    with torch.no_grad():
        want = _oracle_rows(ref, b.x.float().cpu(), b.edge_index.cpu(), rows)
    torch.testing.assert_close(out[rows], want, rtol=2e-2, atol=2e-2)
    assert torch.isfinite(out).all()


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
