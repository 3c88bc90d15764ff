"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Aggregation (gather + per-target reduce, fwd and bwd) is integer-indexed fp32
work done in PyG's CPU edge order, so it must be BITWISE equal to the oracle.
Whole models add GEMMs (different summation order) and are held to the
north-star tolerance: rtol = atol = 1e-5 (fp32) on outputs; gradients, which
chain one more GEMM, to rtol = 1e-4, atol = 1e-5.
"""
import numpy as np
import pytest
import torch

import ngnn
from ngnn import _lib
from ngnn.block import Block, build_csr
from oracle import c_agg, pyg_ref

from test_oracle import MODEL_CASES, _load, load_params
from gradbar import assert_wgrad

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
OUT_TOL = dict(rtol=1e-5, atol=1e-5)
GRAD_TOL = dict(rtol=1e-4, atol=1e-5)


def rand_edges(g, n_src, n_dst, E, order):
    ei = torch.stack([torch.randint(0, n_src, (E,), generator=g),
                      torch.randint(0, n_dst, (E,), generator=g)])
    if order == "dst":
        ei = ei[:, torch.argsort(ei[1], stable=True)]
    elif order == "src":
        ei = ei[:, torch.argsort(ei[0], stable=True)]
    return ei


def gpu_agg(x, ei, reduce, grad=None):
    xd = x.to(DEV).requires_grad_(grad is not None)
    blk = Block(ei.to(DEV), x.shape[0])
    out = ngnn.segment_aggregate(xd, blk, reduce)
    gx = None
    if grad is not None:
        out.backward(grad.to(DEV))
        gx = xd.grad.cpu().numpy()
    torch.cuda.synchronize()
    return out.detach().cpu().numpy(), gx


# ------------------------------------------------------------- CSR build
@pytest.mark.parametrize("order", ["dst", "src", None])
@pytest.mark.parametrize("E", [0, 1, 37, 5000, 200_000])
def test_csr_build_matches_stable_sort(order, E):
    g = torch.Generator().manual_seed(E)
    N = 1000
    ei = rand_edges(g, N, N, E, order)
    keys, vals = ei[1], ei[0]
    csr = build_csr(keys.to(DEV), vals.to(DEV), N, keys_sorted=(order == "dst"))
    perm = np.argsort(keys.numpy(), kind="stable")
    want_col = vals.numpy()[perm].astype(np.int32)
    want_rowptr = np.searchsorted(keys.numpy()[perm], np.arange(N + 1), side="left").astype(np.int32)
    assert np.array_equal(csr.col.cpu().numpy(), want_col)
    assert np.array_equal(csr.rowptr.cpu().numpy(), want_rowptr)


@pytest.mark.parametrize("N,E", [(1, 9), (17, 4097), (70_000, 300_001), (2_449_029, 1_000_003)])
def test_csr_build_unsorted_key_widths(N, E):
    """The unsorted path's in-tree radix passes (4-bit digits, as many as
    ceil(log2 N) needs: 1 .. 6 passes): stable within each key, against
    numpy's stable argsort, up to the products graph's row count."""
    g = torch.Generator().manual_seed(N + E)
    keys = torch.randint(0, N, (E,), generator=g)
    vals = torch.randint(0, N, (E,), generator=g)
    csr = build_csr(keys.to(DEV), vals.to(DEV), N, keys_sorted=False)
    perm = np.argsort(keys.numpy(), kind="stable")
    assert np.array_equal(csr.col.cpu().numpy(), vals.numpy()[perm].astype(np.int32))
    want_rowptr = np.searchsorted(keys.numpy()[perm], np.arange(N + 1), side="left").astype(np.int32)
    assert np.array_equal(csr.rowptr.cpu().numpy(), want_rowptr)


def test_probe_flags_and_index_errors():
    ei = torch.tensor([[0, 1, 2], [2, 1, 0]], device=DEV)
    b = Block(ei, 3)
    assert not b.dst_sorted and b.src_sorted
    with pytest.raises(IndexError):
        Block(torch.tensor([[0, 3], [1, 1]], device=DEV), 3)
    with pytest.raises(IndexError):
        Block(torch.tensor([[0, 1], [1, -1]], device=DEV), 3)


# -------------------------------------------------------- aggregation parity
WIDTHS = [1, 2, 3, 8, 47, 64, 100, 128, 256, 257, 767]


@pytest.mark.parametrize("F", WIDTHS)
@pytest.mark.parametrize("reduce", ["sum", "mean", "max"])
def test_segment_aggregate_bitwise(F, reduce):
    g = torch.Generator().manual_seed(F * 7 + len(reduce))
    N, E = 600, 4000
    ei = rand_edges(g, N, N, E, "dst" if F % 2 else None)
    x = torch.randn(N, F, generator=g)
    go = torch.randn(N, F, generator=g)
    out, gx = gpu_agg(x, ei, reduce, go)
    want = c_agg.agg_fwd(x.numpy(), ei.numpy(), N, reduce)
    assert np.array_equal(out, want)
    want_gx = c_agg.agg_bwd(go.numpy(), ei.numpy(), N, reduce, x.numpy(), want)
    assert np.array_equal(gx, want_gx)


@pytest.mark.parametrize("reduce", ["sum", "mean", "max"])
def test_edge_cases(reduce):
    x = torch.tensor([[1.0, 10.0], [2.0, 20.0], [4.0, 40.0], [8.0, 80.0], [16.0, 160.0]])
    # path, star, duplicate edge, self-loop, isolated node 4; unsorted on purpose
    ei = torch.tensor([[0, 1, 0, 1, 2, 0, 2], [1, 2, 3, 3, 3, 1, 2]])[:, [3, 0, 6, 1, 5, 2, 4]]
    out, gx = gpu_agg(x, ei, reduce, torch.ones(5, 2))
    assert np.array_equal(out, c_agg.agg_fwd(x.numpy(), ei.numpy(), 5, reduce))
    assert np.array_equal(gx, c_agg.agg_bwd(np.ones((5, 2), np.float32), ei.numpy(), 5, reduce,
                                            x.numpy(), out))
    # no edges at all
    out, gx = gpu_agg(x, torch.empty(2, 0, dtype=torch.long), reduce, torch.ones(5, 2))
    assert not out.any() and not gx.any()


def test_max_ties_and_zero_maxima():
    g = torch.Generator().manual_seed(5)
    N = 300
    ei = rand_edges(g, N, N, 3000, "dst")
    x = torch.randn(N, 16, generator=g).relu().round()
    go = torch.randn(N, 16, generator=g)
    out, gx = gpu_agg(x, ei, "max", go)
    xr = x.clone().requires_grad_(True)
    ref = pyg_ref.propagate(xr, ei, "max")
    ref.backward(go)
    assert np.array_equal(out, ref.detach().numpy())
    assert np.array_equal(gx, xr.grad.numpy())


def test_nan_propagation_max():
    x = torch.tensor([[1.0], [float("nan")], [3.0]])
    ei = torch.tensor([[0, 1, 2], [0, 0, 0]])
    out, _ = gpu_agg(x, ei, "max")
    assert np.isnan(out[0, 0]) and out[1, 0] == 0 and out[2, 0] == 0


def test_strided_rows():
    g = torch.Generator().manual_seed(9)
    base = torch.randn(500, 130, generator=g)
    x = base[:, 3:103]  # ld 130, misaligned for float4
    ei = rand_edges(g, 500, 500, 3000, "dst")
    xd = base.to(DEV)[:, 3:103]
    out = ngnn.segment_aggregate(xd, Block(ei.to(DEV), 500), "mean").cpu().numpy()
    assert np.array_equal(out, c_agg.agg_fwd(x.numpy(), ei.numpy(), 500, "mean"))


# ------------------------------------------------- full-size block (metric config)
def test_products_block_full_size_bitwise():
    """A products-like [15,10] bs=1024 block at full size (E ~ 169k): the HIP
    aggregation equals the C oracle bitwise, fwd and bwd, F=100 and 256."""
    from ngnn.loader import sample_block, synthetic_graph
    graph = synthetic_graph("ogbn-products", DEV, seed=0, scale=0.05)
    seeds = graph.train_idx[:1024]
    b = sample_block(graph, seeds, [15, 10], seed=1)
    ei = b.edge_index.cpu()
    N = b.num_nodes
    assert b.edge_index.shape[1] > 100_000
    for F in (100, 256):
        g = torch.Generator().manual_seed(F)
        x = torch.randn(N, F, generator=g)
        go = torch.randn(N, F, generator=g)
        out, gx = gpu_agg(x, ei, "mean", go)
        want = c_agg.agg_fwd(x.numpy(), ei.numpy(), N, "mean")
        assert np.array_equal(out, want)
        assert np.array_equal(gx, c_agg.agg_bwd(go.numpy(), ei.numpy(), N, "mean"))
        # size-independent property: sum-aggregation preserves the column checksum
        s, _ = gpu_agg(x, ei, "sum")
        np.testing.assert_allclose(s.sum(0, dtype=np.float64),
                                   x.numpy()[ei[0].numpy()].sum(0, dtype=np.float64), rtol=1e-4,
                                   atol=1e-2)


# ---------------------------------------------------------- models vs golden
def build_model(kind, kw, aggr):
    if kind == "sage":
        return ngnn.SAGE(aggr=aggr, **kw)
    return ngnn.SimpleGCN(**kw)


@pytest.mark.parametrize("name", sorted(MODEL_CASES))
def test_models_match_reference_golden(golden_dir, name):
    kind, kw, aggr, train = MODEL_CASES[name]
    rec = _load(golden_dir, name)
    m = build_model(kind, kw, aggr)
    load_params(m, rec)
    m.to(DEV).train(train)
    x = torch.from_numpy(rec["x"]).to(DEV).requires_grad_(True)
    ei = torch.from_numpy(rec["edge_index"]).to(DEV)
    out = m(x, ei)
    (out * torch.from_numpy(rec["grad_out"]).to(DEV)).sum().backward()
    torch.testing.assert_close(out.detach().cpu(), torch.from_numpy(rec["out"]), **OUT_TOL)
    torch.testing.assert_close(x.grad.cpu(), torch.from_numpy(rec["grad_x"]), **GRAD_TOL)
    for k, p in m.named_parameters():
        assert_wgrad(p.grad.cpu(), torch.from_numpy(rec["grad/" + k]), msg=f"{name}:{k}")


def test_inference_matches_reference_golden(golden_dir):
    rec = _load(golden_dir, "sage_inference")
    m = ngnn.SAGE(10, 12, 4, 2)
    load_params(m, rec)
    m.to(DEV).eval()

    class B:
        pass

    batches = []
    for i in range(2):
        b = B()
        b.n_id = torch.from_numpy(rec[f"batch{i}/n_id"])
        b.edge_index = torch.from_numpy(rec[f"batch{i}/edge_index"])
        b.batch_size = int(rec[f"batch{i}/batch_size"])
        batches.append(b)
    out = m.inference(torch.from_numpy(rec["x_all"]), batches, DEV)
    assert out.device.type == "cpu"
    torch.testing.assert_close(out, torch.from_numpy(rec["out"]), **OUT_TOL)


def test_training_step_matches_oracle():
    """Two Adam steps of the metric model (100->256->47) on a sampled block:
    parameters after the steps match the oracle's within tolerance."""
    from ngnn.loader import sample_block, synthetic_graph
    graph = synthetic_graph("ogbn-products", DEV, seed=1, scale=0.01)
    b = sample_block(graph, graph.train_idx[:256], [15, 10], seed=3)
    torch.manual_seed(0)
    ref = pyg_ref.SAGE(100, 256, 47, 2, dropout=0.0)
    mine = ngnn.SAGE(100, 256, 47, 2, dropout=0.0)
    mine.load_state_dict(ref.state_dict())
    mine.to(DEV)
    o_ref = torch.optim.Adam(ref.parameters(), lr=1e-3)
    o_mine = torch.optim.Adam(mine.parameters(), lr=1e-3)
    xc, eic, yc = b.x.cpu(), b.edge_index.cpu(), b.y.cpu()
    for _ in range(2):
        l_ref = pyg_ref.train_step(ref, o_ref, xc, eic, yc, b.batch_size)
        l_mine = pyg_ref.train_step(mine, o_mine, b.x, b.edge_index, b.y, b.batch_size)
        assert abs(float(l_ref) - float(l_mine)) < 1e-5
    for (k, p), (_, q) in zip(mine.state_dict().items(), ref.state_dict().items()):
        torch.testing.assert_close(p.cpu(), q, rtol=1e-4, atol=1e-5, msg=k)


@pytest.mark.parametrize("module", ["sage", "gcn"])
def test_bf16_model_matches_fp32_oracle(module):
    """A bf16 model (BASELINE config #3 asks for bf16): bf16 inputs and
    parameters, fp32 arithmetic inside -- equal to the fp32 oracle run on the
    same bf16-rounded values up to the bf16 rounding of the logits (rtol 1e-2,
    the bar SURVEY §8c sets for bf16), gradients in bf16."""
    import ngnn
    from ngnn.loader import sample_block, synthetic_graph
    graph = synthetic_graph("ogbn-products", DEV, seed=5, scale=0.005)
    b = sample_block(graph, graph.train_idx[:64], [6, 4, 3], seed=2)
    torch.manual_seed(3)
    if module == "sage":
        mine = ngnn.SAGE(100, 64, 47, 3, dropout=0.5).eval()
        ref = pyg_ref.SAGE(100, 64, 47, 3, dropout=0.5).eval()
    else:
        mine = ngnn.SimpleGCN(100, 64, 47, 3, dropout=0.5).eval()
        ref = pyg_ref.SimpleGCN(100, 64, 47, 3, dropout=0.5).eval()
    mine = mine.to(DEV).to(torch.bfloat16)
    ref.load_state_dict({k: v.float().cpu() for k, v in mine.state_dict().items()})
    xb = b.x.to(torch.bfloat16).requires_grad_(True)
    out = mine(xb, b.edge_index)
    assert out.dtype == torch.bfloat16
    out.float().square().sum().backward()
    assert xb.grad.dtype == torch.bfloat16
    assert all(p.grad.dtype == torch.bfloat16 for p in mine.parameters())
    xr = xb.detach().float().cpu().requires_grad_(True)
    want = ref(xr, b.edge_index.cpu())
    # bf16 logits (and, through the per-conv GCN path, bf16 activations between
    # layers): compare in norm, 1e-2 relative
    err = (out.float().cpu() - want.detach()).norm() / want.detach().norm()
    assert err < 1e-2, float(err)
