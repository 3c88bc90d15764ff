"""GPU parity of the two-layer weight-stationary forward (ngnn_sage2_fwd,
csrc/ngnn_fwd2.hip): SAGE(K0, 256, F1) on a NeighborLoader-shaped block,
against the CPU oracle (oracle/pyg_ref.py, the PyG 2.5.1 op sequence of
sage.py:33-39).

* h (layer 0's output after ReLU / dropout), the logits of every row and the
  saved layer-0 aggregate, at the fp32 bars (outputs rtol = atol = 1e-5); the
  aggregate bitwise against the C restatement (oracle/seg_agg.c);
* train mode with the hash dropout in bit mode (p = 0.5) and byte mode
  (p = 0.2), masks rebuilt on the host;
* the H2 arithmetic's scaling at extreme magnitudes (rows of 1e6 and 1e-8,
  all-zero rows, weights of 1e3) -- relative to the oracle;
* ragged shapes: N not a multiple of 16, tiny blocks, every row with
  in-edges, rows without in-edges inside the edge tiles;
* the stack's backward on the new forward's saved tensors (every gradient).
"""
import pytest
import torch
import torch.nn.functional as F

import ngnn
from ngnn import fused
from ngnn.block import Block
from oracle import c_agg, pyg_ref

from test_gpu_fused import GRAD, OUT, _MaskedSAGE, dropout_keep, dropout_scale
from gradbar import assert_wgrad

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _block(seed, N, n_active, deg_max=15, zero_rows=()):
    """Target-sorted edges into rows < n_active (deg 0..deg_max, some rows
    with none), sources anywhere -- the NeighborLoader layout."""
    g = torch.Generator().manual_seed(seed)
    deg = torch.randint(0, deg_max + 1, (n_active,), generator=g)
    for r in zero_rows:
        if r < n_active:
            deg[r] = 0
    dst = torch.repeat_interleave(torch.arange(n_active), deg)
    src = torch.randint(0, N, (dst.numel(),), generator=g)
    ei = torch.stack([src, dst])
    blk = Block(ei.to(DEV), N)
    blk.n_active = n_active
    return ei, blk


def _params(K0, H, F1, seed, wscale=1.0):
    torch.manual_seed(seed)
    ref = pyg_ref.SAGE(K0, H, F1, 2, dropout=0.5)
    if wscale != 1.0:
        with torch.no_grad():
            for p in ref.parameters():
                p.mul_(wscale)
    return ref


def _run_fwd2(x, blk, ref, reduce, p, seed):
    params = [ref.convs[0].lin_l.weight, ref.convs[0].lin_l.bias, ref.convs[0].lin_r.weight,
              ref.convs[1].lin_l.weight, ref.convs[1].lin_l.bias, ref.convs[1].lin_r.weight]
    params = [q.detach().to(DEV) for q in params]
    xd = x.to(DEV)
    assert fused.sage2_ok(xd, blk, reduce, params, False)
    h, out, agg0, partial = fused.sage2_forward(xd, blk, reduce, params, p, seed, None)
    assert not partial
    return h.cpu(), out.cpu(), agg0.cpu()


def _oracle(x, ei, ref, reduce, p, seed, N, H):
    for c in ref.convs:
        c.aggr = reduce
    h = ref.convs[0](x, ei).relu()
    if p > 0:
        h = h * dropout_keep(seed, N, H, p).float() * dropout_scale(p)
    return h, ref.convs[1](h, ei)


@pytest.mark.parametrize("K0,F1", [(100, 47), (128, 40), (100, 48), (124, 33), (100, 45)])
@pytest.mark.parametrize("reduce", ["mean", "sum"])
@pytest.mark.parametrize("p", [0.0, 0.5, 0.2])
def test_fwd2_matches_oracle(K0, F1, reduce, p):
    N, n_act, H = 3000 + K0 % 7, 700, 256
    ei, blk = _block(K0 + F1, N, n_act, zero_rows=(3, 17, 640))
    g = torch.Generator().manual_seed(K0 * F1)
    x = torch.randn(N, K0, generator=g)
    ref = _params(K0, H, F1, 1)
    seed = 1234567 + K0
    h, out, agg0 = _run_fwd2(x, blk, ref, reduce, p, seed)
    with torch.no_grad():
        h_r, out_r = _oracle(x, ei, ref, reduce, p, seed, N, H)
    torch.testing.assert_close(h, h_r, **OUT)
    torch.testing.assert_close(out, out_r, **OUT)
    # the saved aggregate: bitwise the C restatement, rows of the edge tiles
    want = c_agg.agg_fwd(x.numpy(), ei.numpy(), N, reduce)
    rows = -(-n_act // 16) * 16
    assert torch.equal(agg0[:rows], torch.from_numpy(want[:rows]))


@pytest.mark.parametrize("N,n_act", [(5, 5), (17, 17), (16, 3), (33, 1), (1000, 1000), (1001, 0)])
def test_fwd2_ragged_blocks(N, n_act):
    K0, H, F1 = 100, 256, 47
    ei, blk = _block(N, N, n_act, deg_max=6)
    x = torch.randn(N, K0, generator=torch.Generator().manual_seed(N))
    ref = _params(K0, H, F1, 2)
    h, out, _ = _run_fwd2(x, blk, ref, "mean", 0.5, 77)
    with torch.no_grad():
        h_r, out_r = _oracle(x, ei, ref, "mean", 0.5, 77, N, H)
    torch.testing.assert_close(h, h_r, **OUT)
    torch.testing.assert_close(out, out_r, **OUT)


@pytest.mark.parametrize("p", [0.0, 0.5, 0.25])
def test_fwd2_many_tiles_per_workgroup(p):
    """~12 tiles per workgroup (the blocks above give each workgroup one):
    every step of the software pipeline -- both parts-buffer parities, the
    edge phase and the plain phase, the reduce of the previous tile -- against
    the oracle, and two launches bit-identical (a cross-wave race or a missed
    register hazard shows up as scattered wrong rows that move between runs)."""
    N, n_act, K0, H, F1 = 48_000 + 13, 9_000, 100, 256, 47
    ei, blk = _block(31, N, n_act, deg_max=10, zero_rows=(5, 4096, 8191))
    x = torch.randn(N, K0, generator=torch.Generator().manual_seed(32))
    ref = _params(K0, H, F1, 4)
    seed = 99 + int(100 * p)
    h, out, _ = _run_fwd2(x, blk, ref, "mean", p, seed)
    h2, out2, _ = _run_fwd2(x, blk, ref, "mean", p, seed)
    assert torch.equal(h, h2) and torch.equal(out, out2)
    with torch.no_grad():
        h_r, out_r = _oracle(x, ei, ref, "mean", p, seed, N, H)
    torch.testing.assert_close(h, h_r, **OUT)
    torch.testing.assert_close(out, out_r, **OUT)


@pytest.mark.parametrize("xscale,wscale", [(1e6, 1.0), (1e-8, 1.0), (1.0, 1e3), (1e4, 1e-3)])
def test_fwd2_scaling_extremes(xscale, wscale):
    """Power-of-two scaling per row / per matrix keeps the fp16 parts in
    range: the result tracks the oracle relatively at any magnitude; an
    all-zero row gives exactly the bias path."""
    N, n_act, K0, H, F1 = 900, 300, 100, 256, 47
    ei, blk = _block(5, N, n_act)
    x = torch.randn(N, K0, generator=torch.Generator().manual_seed(9)) * xscale
    x[10] = 0.0      # a zero row with in-edges
    x[500] = 0.0     # a zero row without
    x[501, :50] *= 1e-12  # one row with a huge dynamic range
    ref = _params(K0, H, F1, 3, wscale)
    h, out, _ = _run_fwd2(x, blk, ref, "mean", 0.0, 0)
    with torch.no_grad():
        h_r, out_r = _oracle(x, ei, ref, "mean", 0.0, 0, N, H)
    tol_h = dict(rtol=1e-5, atol=1e-5 * float(h_r.abs().max()))
    tol_o = dict(rtol=1e-5, atol=1e-5 * float(out_r.abs().max()))
    torch.testing.assert_close(h, h_r, **tol_h)
    torch.testing.assert_close(out, out_r, **tol_o)


@pytest.mark.parametrize("train", [False, True])
@pytest.mark.parametrize("aggr", ["mean", "sum"])
def test_fwd2_stack_backward_matches_oracle(train, aggr):
    """The whole stack (ngnn.SAGE) on a sampled block routes through
    ngnn_sage2_fwd; its backward on the saved h / aggregate matches the
    oracle's gradients (input, every parameter)."""
    from ngnn.loader import sample_block, synthetic_graph
    graph = synthetic_graph("ogbn-products", DEV, seed=2, scale=0.01)
    b = sample_block(graph, graph.train_idx[:256], [15, 10], seed=4)
    N = b.num_nodes
    torch.manual_seed(11)
    mine = ngnn.SAGE(100, 256, 47, 2, dropout=0.5, aggr=aggr).to(DEV).train(train)
    seed = None
    if train:
        torch.manual_seed(99)
        seed = int(torch.randint(0, 2**62, (1,)).item())
        torch.manual_seed(99)
    calls = []
    orig = fused.sage2_forward

    def spy(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    fused.sage2_forward = spy
    fused._debug_acts = []
    try:
        x = b.x.clone().requires_grad_(True)
        out = mine(x, b.edge_index)
        F.cross_entropy(out[:b.batch_size], b.y[:b.batch_size]).backward()
        hid = [a.cpu() for a in fused._debug_acts[-1]]
    finally:
        fused.sage2_forward = orig
        fused._debug_acts = None
    assert calls, "the stack did not take ngnn_sage2_fwd"
    # (ReLU kinks: the GPU's decision where fp32 order decides, _MaskedSAGE)
    ref = _MaskedSAGE(100, 256, 47, 2, dropout=0.5, aggr=aggr, gpu_hidden=hid,
                      masks=[dropout_keep(seed, N, 256, 0.5).float()] if train else None)
    ref.train(train)
    ref.load_state_dict({k: v.cpu() for k, v in mine.state_dict().items()})
    xr = b.x.cpu().clone().requires_grad_(True)
    out_r = ref(xr, b.edge_index.cpu())
    F.cross_entropy(out_r[:b.batch_size], b.y[:b.batch_size].cpu()).backward()
    torch.testing.assert_close(out.detach().cpu(), out_r.detach(), **OUT)
    torch.testing.assert_close(x.grad.cpu(), xr.grad, **GRAD)
    for (k, p), (_, q) in zip(mine.named_parameters(), ref.named_parameters()):
        assert_wgrad(p.grad.cpu(), q.grad, msg=k)


def test_fwd2_equals_per_layer_path_within_bars():
    """The two forwards (weight-stationary H2 vs per-layer split-bf16) agree
    within the fp32 bar on a sampled products block; both are deterministic."""
    from ngnn.loader import sample_block, synthetic_graph
    graph = synthetic_graph("ogbn-products", DEV, seed=3, scale=0.01)
    b = sample_block(graph, graph.train_idx[:512], [15, 10], seed=5)
    torch.manual_seed(0)
    mine = ngnn.SAGE(100, 256, 47, 2).to(DEV).eval()
    with torch.no_grad():
        a1 = mine(b.x, b.edge_index)
        a2 = mine(b.x, b.edge_index)
        fused._use_fwd2 = False
        try:
            p1 = mine(b.x, b.edge_index)
        finally:
            fused._use_fwd2 = True
    assert torch.equal(a1, a2)
    torch.testing.assert_close(a1, p1, **OUT)
