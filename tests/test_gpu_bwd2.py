"""GPU parity of the two-layer backward (ngnn_sage2_bwd, csrc/ngnn_bwd2.hip):
every weight gradient of SAGE(K0, 256, F1) against a float64 restatement of
the reference's autograd (sage.py:33-39 under loss.backward(): per layer
dW_l = dz^T agg(h_in), dW_r = dz^T h_in, db = sum dz; the ReLU / dropout
backward of the hidden layer), on NeighborLoader-shaped blocks:

* the top-layer gradient dy nonzero on the seed rows < R only, h nonzero on
  a random subset (the ReLU / dropout mask), agg0 the C restatement's
  aggregate (oracle/seg_agg.c), rows without in-edges among rows < R';
* mean and sum, several F1 / K0, the fused x[n_id] gather (x = table rows);
* the workspace invariant (g zero again on return: a second call repeats);
* the stack backward through the graph slot uses it (spy) and matches the
  per-layer backward within the bars.
Bar: tests/gradbar.py (max|g - g_ref| <= 1e-5 max|g_ref| per tensor), as every
fp32 weight-gradient test.
"""
import numpy as np
import pytest
import torch

from ngnn import _lib
from oracle import c_agg

from gradbar import assert_wgrad

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _case(seed, N, R, Rn, K0, F1, xr=False, deg_max=15):
    """A block whose rows < Rn have in-edges (some with none); sources of
    edges into rows < R below Rn, the others anywhere; dy rows < R; h rows
    < Rn with about half of them zero."""
    g = torch.Generator().manual_seed(seed)
    deg = torch.randint(0, deg_max + 1, (Rn,), generator=g)
    deg[:: 7] = 0
    dst = torch.repeat_interleave(torch.arange(Rn), deg)
    # R' is a bound: the sources of edges into the seed rows are rows < R'
    src = torch.where(dst < R, torch.randint(0, Rn, (dst.numel(),), generator=g),
                      torch.randint(0, N, (dst.numel(),), generator=g))
    ei = torch.stack([src, dst])
    rowptr = torch.zeros(N + 1, dtype=torch.int32)
    rowptr[1:Rn + 1] = torch.cumsum(deg, 0).to(torch.int32)
    rowptr[Rn + 1:] = rowptr[Rn]
    col = torch.zeros(max(src.numel(), 1), dtype=torch.int32)  # (a non-null pointer for no edges)
    col[:src.numel()] = src.to(torch.int32)
    dy = torch.zeros(N, F1)
    dy[:R] = torch.randn(R, F1, generator=g) * 1e-3
    h = torch.relu(torch.randn(N, 256, generator=g)) * (torch.rand(N, 256, generator=g) > 0.3).float() * 2.0
    h[Rn:] = float("nan")  # never read
    if xr:
        table = torch.randn(3 * N + 5, K0, generator=g)
        xrow = torch.randint(0, table.size(0), (N,), generator=g)
        x = table[xrow]
    else:
        table, xrow = None, None
        x = torch.randn(N, K0, generator=g)
    agg0 = torch.from_numpy(c_agg.agg_fwd(x.numpy(), ei.numpy(), N, "mean"))
    wl1 = torch.randn(F1, 256, generator=g) * 0.05
    wr1 = torch.randn(F1, 256, generator=g) * 0.05
    return dict(ei=ei, rowptr=rowptr, col=col, dy=dy, h=h, x=x, table=table, xrow=xrow, agg0=agg0,
                wl1=wl1, wr1=wr1)


def _reference(c, R, Rn, reduce, yscale):
    """float64: the per-layer autograd formulas of the reference."""
    ei = c["ei"].long()
    src, dst = ei[0], ei[1]
    N = c["dy"].size(0)
    dy = c["dy"].double()
    h = c["h"][:Rn].double()
    deg = torch.bincount(dst, minlength=N).double()
    w = torch.ones(dst.numel(), dtype=torch.float64)
    if reduce == "mean":
        w = w / deg[dst].clamp(min=1)
    # top layer: agg(h) over rows < R, then the input gradient of h
    aggh = torch.zeros(N, 256, dtype=torch.float64)
    hh = torch.nan_to_num(c["h"].double(), nan=0.0)
    aggh.index_add_(0, dst, hh[src] * w[:, None])
    dWl1 = dy[:R].T @ aggh[:R]
    dWr1 = dy[:R].T @ hh[:R]
    db1 = dy[:R].sum(0)
    dh = dy @ c["wr1"].double()
    gsc = torch.zeros(N, dy.size(1), dtype=torch.float64)
    m = dst < R
    gsc.index_add_(0, src[m], dy[dst[m]] * w[m][:, None])
    dh = dh + gsc @ c["wl1"].double()
    dz0 = (dh[:Rn] * (h > 0).double()) * yscale
    x = c["x"][:Rn].double()
    agg0 = c["agg0"][:Rn].double()
    return dict(dWl1=dWl1, dbl1=db1, dWr1=dWr1, dWl0=dz0.T @ agg0, dbl0=dz0.sum(0), dWr0=dz0.T @ x)


def _run(c, R, Rn, reduce, yscale, ws=None):
    lib = _lib.load()
    N, K0 = c["x"].shape
    F1 = c["dy"].size(1)
    d = {k: (v.to(DEV) if isinstance(v, torch.Tensor) else v) for k, v in c.items()}
    out = dict(dWl1=torch.empty(F1, 256, device=DEV), dbl1=torch.empty(F1, device=DEV),
               dWr1=torch.empty(F1, 256, device=DEV), dWl0=torch.empty(256, K0, device=DEV),
               dbl0=torch.empty(256, device=DEV), dWr0=torch.empty(256, K0, device=DEV))
    bounds = torch.tensor([R, Rn], dtype=torch.int32, device=DEV)
    if ws is None:
        ws = torch.zeros(lib.ngnn_sage2_bwd_workspace_bytes(N, K0, F1), dtype=torch.uint8, device=DEV)
    xr = d["table"] is not None
    x = d["table"] if xr else d["x"]
    xrow = d["xrow"] if xr else None
    rc = lib.ngnn_sage2_bwd(
        _lib.ptr(d["dy"]), F1, F1, _lib.ptr(d["wl1"]), _lib.ptr(d["wr1"]), 256, _lib.ptr(d["h"]), 256,
        yscale, _lib.ptr(x), None, _lib.ptr(xrow), None, x.size(0) if xr else 0, K0, K0,
        _lib.ptr(d["agg0"]), K0, _lib.ptr(d["rowptr"]), _lib.ptr(d["col"]), N,
        bounds.data_ptr(), bounds.data_ptr() + 4, _lib.REDUCE[reduce],
        *(_lib.ptr(out[k]) for k in ("dWl1", "dbl1", "dWr1", "dWl0", "dbl0", "dWr0")), None, None,
        _lib.ptr(ws), ws.numel(), _lib.stream_handle(DEV))
    assert rc == _lib.OK, rc
    torch.cuda.synchronize()
    return {k: v.cpu() for k, v in out.items()}, ws


@pytest.mark.parametrize("K0,F1", [(100, 47), (128, 40), (100, 33), (64, 48)])
@pytest.mark.parametrize("reduce", ["mean", "sum"])
def test_bwd2_matches_reference(K0, F1, reduce):
    N, R, Rn = 3000, 300, 1500
    c = _case(K0 + F1, N, R, Rn, K0, F1)
    ys = 2.0
    got, ws = _run(c, R, Rn, reduce, ys)
    want = _reference(c, R, Rn, reduce, ys)
    for k in want:
        assert_wgrad(got[k].double(), want[k], msg=k)
    # the workspace's g part is zero again (it sits after the 64 slabs), so
    # a second call on it repeats the first within the bars (the g atomics'
    # order varies run to run: not bitwise)
    slab = 64 * (512 * K0 + 256 + 512 * F1 + F1) * 4
    goff = (slab + 255) // 256 * 256
    assert int(ws[goff:].count_nonzero()) == 0
    again, _ = _run(c, R, Rn, reduce, ys, ws=ws)
    for k in want:
        assert_wgrad(again[k].double(), want[k], msg=k)


@pytest.mark.parametrize("N,R,Rn", [(17, 3, 9), (40, 40, 40), (5000, 1024, 4700), (2000, 1, 1)])
def test_bwd2_ragged_bounds(N, R, Rn):
    c = _case(N, N, R, Rn, 100, 47)
    got, _ = _run(c, R, Rn, "mean", 1.25)
    want = _reference(c, R, Rn, "mean", 1.25)
    for k in want:
        assert_wgrad(got[k].double(), want[k], msg=k)


def test_bwd2_fused_row_gather():
    """x rows through n_id (the zero-copy slot's fused gather)."""
    N, R, Rn = 2500, 256, 1200
    c = _case(7, N, R, Rn, 100, 47, xr=True)
    got, _ = _run(c, R, Rn, "mean", 2.0)
    want = _reference(c, R, Rn, "mean", 2.0)
    for k in want:
        assert_wgrad(got[k].double(), want[k], msg=k)


def test_bwd2_headline_size_against_float64():
    """A full products-sized block's bounds (R = 1024 seeds, R' ~ 16 k) with
    the C restatement's aggregate: every gradient within the bars."""
    N, R, Rn = 150_000, 1024, 16_000
    c = _case(11, N, R, Rn, 100, 47, deg_max=15)
    got, _ = _run(c, R, Rn, "mean", 2.0)
    want = _reference(c, R, Rn, "mean", 2.0)
    for k in want:
        assert_wgrad(got[k].double(), want[k], msg=k)


def test_stack_backward_routes_through_bwd2():
    """The graph slot's step (seed_cross_entropy: the loss reads rows < B)
    takes ngnn_sage2_bwd; its gradients match the per-layer backward's."""
    import ngnn
    from ngnn import fused
    from ngnn.graphs import GraphedTrainStep, slot_size
    from ngnn.loader import sample_block, synthetic_graph
    from ngnn.optim import Adam
    graph = synthetic_graph("ogbn-products", DEV, seed=5, scale=0.02)
    b = sample_block(graph, graph.train_idx[:512], [15, 10], seed=9)
    grads = []
    for use in (True, False):
        torch.manual_seed(0)
        model = ngnn.SAGE(100, 256, 47, 2, dropout=0.5).to(DEV).train()
        opt = Adam(model.parameters(), lr=1e-3)
        n_cap, e_cap = slot_size(512, [15, 10])
        step = GraphedTrainStep(model, opt, 512, n_cap, e_cap, 100, DEV)
        calls = []
        orig = fused.sage2_backward

        def spy(*a, **k):
            calls.append(1)
            return orig(*a, **k)

        fused.sage2_backward, fused._use_bwd2 = spy, use
        try:
            step.capture(b.x, b.edge_index, b.y)
            step(b.x, b.edge_index, b.y)
            torch.cuda.synchronize()
        finally:
            fused.sage2_backward, fused._use_bwd2 = orig, True
        assert bool(calls) == use
        grads.append({k: p.grad.detach().cpu().clone() for k, p in model.named_parameters()})
    for k in grads[0]:
        assert_wgrad(grads[0][k], grads[1][k], msg=k)


def test_eager_reference_loop_routes_through_bwd2():
    """The reference loop on ngnn's modules without a graph slot (INTEGRATION
    Option B: out = model(x, ei)[:bs], F.cross_entropy, backward; x needs no
    gradient) takes ngnn_sage2_bwd with row bounds from dout on the device;
    its gradients match the per-layer backward's and the oracle's."""
    import torch.nn.functional as F

    import ngnn
    from ngnn import fused
    from ngnn.loader import sample_block, synthetic_graph
    from test_gpu_fused import _MaskedSAGE, dropout_keep
    graph = synthetic_graph("ogbn-products", DEV, seed=6, scale=0.02)
    b = sample_block(graph, graph.train_idx[:512], [15, 10], seed=3)
    grads, calls, hid = [], [], None
    orig = fused.sage2_backward

    def spy(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    for use in (True, False):
        torch.manual_seed(0)
        model = ngnn.SAGE(100, 256, 47, 2, dropout=0.5).to(DEV).train()
        init = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
        torch.manual_seed(42)
        seed = int(torch.randint(0, 2**62, (1,)).item())
        torch.manual_seed(42)
        fused.sage2_backward, fused._use_bwd2, fused._debug_acts = spy, use, []
        try:
            out = model(b.x, b.edge_index)[:b.batch_size]
            F.cross_entropy(out, b.y[:b.batch_size]).backward()
            hid = [a.cpu() for a in fused._debug_acts[-1]]
        finally:
            fused.sage2_backward, fused._use_bwd2, fused._debug_acts = orig, True, None
        assert bool(calls) == use
        calls.clear()
        grads.append({k: p.grad.detach().cpu().clone() for k, p in model.named_parameters()})
    ref = _MaskedSAGE(100, 256, 47, 2, dropout=0.5, gpu_hidden=hid,
                      masks=[dropout_keep(seed, b.num_nodes, 256, 0.5).float()])
    ref.load_state_dict(init)
    F.cross_entropy(ref(b.x.cpu(), b.edge_index.cpu())[:b.batch_size], b.y[:b.batch_size].cpu()).backward()
    for k, q in ref.named_parameters():
        assert_wgrad(grads[0][k], q.grad, msg=f"bwd2:{k}")
        assert_wgrad(grads[1][k], q.grad, msg=f"per-layer:{k}")


@pytest.mark.parametrize("train", [True, False])
def test_eager_cpp_node_matches_python_node(train):
    """The eager step's C++ autograd node (csrc/ngnn_eager.cpp) makes the
    Python node's launches: the same logits bit for bit and the same weight
    gradients (within the bar: the backward's atomics), train (dropout) and
    eval; it is the node that ran."""
    import torch.nn.functional as F

    import ngnn
    from ngnn import _eager, fused
    from ngnn.loader import sample_block, synthetic_graph
    if _eager.load() is None:
        pytest.fail("ngnn_eager.so not built (__graft_entry__.build())")
    graph = synthetic_graph("ogbn-products", DEV, seed=8, scale=0.02)
    b = sample_block(graph, graph.train_idx[:512], [15, 10], seed=4)
    outs, grads = [], []
    for use in (True, False):
        torch.manual_seed(0)
        model = ngnn.SAGE(100, 256, 47, 2, dropout=0.5).to(DEV).train(train)
        torch.manual_seed(42)
        n0 = fused.eager_ext_calls
        fused._use_eager_ext = use
        try:
            for _ in range(2):  # (twice: the second backward accumulates)
                out = model(b.x, b.edge_index)[:b.batch_size]
                F.cross_entropy(out, b.y[:b.batch_size]).backward()
        finally:
            fused._use_eager_ext = True
        assert (fused.eager_ext_calls - n0 == 2) == use
        outs.append(out.detach().cpu())
        grads.append({k: p.grad.detach().cpu().clone() for k, p in model.named_parameters()})
    assert torch.equal(outs[0], outs[1])
    for k in grads[0]:
        assert_wgrad(grads[0][k], grads[1][k], msg=k)
