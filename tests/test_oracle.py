"""CPU tests of the oracle: hand-computed known answers, C restatement vs the
torch restatement (bitwise), and both against the golden fixtures produced by
executing the reference's own sage.py / convolution.py (tests/golden)."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import c_agg, pyg_ref


def _ei(pairs):
    return torch.tensor(pairs, dtype=torch.long).t().contiguous()


# ---------------------------------------------------------------- known answers
@pytest.mark.parametrize("impl", ["torch", "c"])
def test_kat_path_star_isolated_duplicate_selfloop(impl):
    # nodes: 0..4 ; node 4 isolated (no in-edges)
    x = torch.tensor([[1.0, 10.0], [2.0, 20.0], [4.0, 40.0], [8.0, 80.0], [16.0, 160.0]])
    # 0->1, 1->2 (path), 0->3, 1->3, 2->3 (star into 3), duplicate 0->1, self loop 2->2
    ei = _ei([(0, 1), (1, 2), (0, 3), (1, 3), (2, 3), (0, 1), (2, 2)])
    want = {
        "sum": [[0, 0], [2, 20], [6, 60], [7, 70], [0, 0]],
        "mean": [[0, 0], [1, 10], [3, 30], [7 / 3, 70 / 3], [0, 0]],
        "max": [[0, 0], [1, 10], [4, 40], [4, 40], [0, 0]],
    }
    for red, w in want.items():
        if impl == "torch":
            got = pyg_ref.propagate(x, ei, red)
        else:
            got = torch.from_numpy(c_agg.agg_fwd(x.numpy(), ei.numpy(), 5, red))
        torch.testing.assert_close(got, torch.tensor(w, dtype=torch.float32), rtol=0, atol=1e-6)


def test_kat_empty_edges():
    x = torch.randn(4, 3)
    ei = torch.empty(2, 0, dtype=torch.long)
    for red in ["sum", "mean", "max"]:
        assert torch.equal(pyg_ref.propagate(x, ei, red), torch.zeros(4, 3))
        assert np.array_equal(c_agg.agg_fwd(x.numpy(), ei.numpy(), 4, red), np.zeros((4, 3), np.float32))


def test_kat_max_tie_rule():
    # three sources all 0 into node 0, max = 0: the zero `self` counts as a tie,
    # so each source gets g/4 (torch scatter_reduce amax backward).
    x = torch.tensor([[0.0, 1.0], [0.0, 1.0], [0.0, 3.0], [5.0, 5.0]], requires_grad=True)
    ei = _ei([(0, 3), (1, 3), (2, 3)])
    out = pyg_ref.propagate(x, ei, "max")
    out.backward(torch.ones_like(out))
    want = torch.tensor([[0.25, 0.0], [0.25, 0.0], [0.25, 1.0], [0.0, 0.0]])
    torch.testing.assert_close(x.grad, want)
    gx = c_agg.agg_bwd(np.ones((4, 2), np.float32), ei.numpy(), 4, "max", x.detach().numpy(),
                       out.detach().numpy())
    assert np.array_equal(gx, want.numpy())


def test_kat_mean_backward_hand():
    # dst 2 has in-edges from 0 and 1 (deg 2), dst 1 from 0 (deg 1)
    ei = _ei([(0, 2), (1, 2), (0, 1)])
    g = np.array([[1, 1], [3, 5], [2, 4]], np.float32)
    gx = c_agg.agg_bwd(g, ei.numpy(), 3, "mean")
    # x0 <- g2/2 + g1/1 ; x1 <- g2/2 ; x2 <- 0
    assert np.array_equal(gx, np.array([[4, 7], [1, 2], [0, 0]], np.float32))


# ------------------------------------------------ C restatement vs torch, bitwise
@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("reduce", ["sum", "mean", "max"])
@pytest.mark.parametrize("order", ["dst", "src", None])
def test_c_matches_torch_bitwise(seed, reduce, order):
    g = torch.Generator().manual_seed(seed)
    N, F, E = 257, 19 + seed, 1500
    ei = torch.randint(0, N, (2, E), generator=g)
    if order == "dst":
        ei = ei[:, torch.argsort(ei[1], stable=True)]
    elif order == "src":
        ei = ei[:, torch.argsort(ei[0], stable=True)]
    x = torch.randn(N, F, generator=g)
    if reduce == "max" and seed == 2:
        x = x.relu().round()  # many ties incl. zero maxima
    xr = x.clone().requires_grad_(True)
    out = pyg_ref.propagate(xr, ei, reduce)
    go = torch.randn(out.shape, generator=g)
    out.backward(go)
    o = c_agg.agg_fwd(x.numpy(), ei.numpy(), N, reduce)
    gx = c_agg.agg_bwd(go.numpy(), ei.numpy(), N, reduce, x.numpy(), out.detach().numpy())
    assert np.array_equal(o, out.detach().numpy())
    assert np.array_equal(gx, xr.grad.numpy())


# ---------------------------------------------------------- golden fixtures
def _load(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, name + ".npz"), allow_pickle=False))


MODEL_CASES = {
    "sage_mean_block": ("sage", dict(in_size=100, hidden_size=32, out_size=47, num_layers=2), "mean", False),
    "sage_mean_3layer_unsorted": ("sage", dict(in_size=24, hidden_size=40, out_size=7, num_layers=3), "mean", False),
    "sage_mean_srcsorted": ("sage", dict(in_size=128, hidden_size=64, out_size=40, num_layers=2), "mean", False),
    "sage_mean_bn_train": ("sage", dict(in_size=16, hidden_size=32, out_size=5, num_layers=2, dropout=0.0, use_bn=True), "mean", True),
    "gcn_2layer": ("gcn", dict(in_size=20, hidden_size=32, out_size=6, num_layers=2), None, False),
    "gcn_3layer_unsorted": ("gcn", dict(in_size=12, hidden_size=16, out_size=16, num_layers=3), None, False),
    "sage_max_block": ("sage", dict(in_size=767, hidden_size=16, out_size=10, num_layers=2), "max", False),
    "sage_max_ties": ("sage", dict(in_size=8, hidden_size=8, out_size=3, num_layers=2), "max", False),
}


def build_oracle_model(kind, kw, aggr):
    if kind == "sage":
        return pyg_ref.SAGE(aggr=aggr, **kw)
    return pyg_ref.SimpleGCN(**kw)


def load_params(model, rec):
    sd = {k[len("param/"):]: torch.from_numpy(v) for k, v in rec.items() if k.startswith("param/")}
    model.load_state_dict(sd)
    return sd


def test_golden_files_present(golden_dir):
    names = {os.path.basename(p)[:-4] for p in glob.glob(os.path.join(golden_dir, "*.npz"))}
    assert set(MODEL_CASES) | {"sage_inference"} <= names


@pytest.mark.parametrize("name", sorted(MODEL_CASES))
def test_oracle_reproduces_reference_golden(golden_dir, name):
    kind, kw, aggr, train = MODEL_CASES[name]
    rec = _load(golden_dir, name)
    m = build_oracle_model(kind, kw, aggr)
    sd = load_params(m, rec)
    # state-dict contract (key names, shapes) of the reference model
    assert list(sd) == list(m.state_dict())
    m.train(train)
    x = torch.from_numpy(rec["x"]).requires_grad_(True)
    ei = torch.from_numpy(rec["edge_index"])
    out = m(x, ei)
    (out * torch.from_numpy(rec["grad_out"])).sum().backward()
    # same ops in the same order on the same CPU -> bitwise
    assert np.array_equal(out.detach().numpy(), rec["out"]), name
    assert np.array_equal(x.grad.numpy(), rec["grad_x"]), name
    for k, p in m.named_parameters():
        assert np.array_equal(p.grad.numpy(), rec["grad/" + k]), (name, k)


def test_oracle_inference_golden(golden_dir):
    rec = _load(golden_dir, "sage_inference")
    m = pyg_ref.SAGE(10, 12, 4, 2).eval()
    load_params(m, rec)

    class B:
        pass

    batches = []
    for i in range(2):
        b = B()
        b.n_id = torch.from_numpy(rec[f"batch{i}/n_id"])
        b.edge_index = torch.from_numpy(rec[f"batch{i}/edge_index"])
        b.batch_size = int(rec[f"batch{i}/batch_size"])
        batches.append(b)
    with torch.no_grad():
        out = m.inference(torch.from_numpy(rec["x_all"]), batches, "cpu")
    assert np.array_equal(out.numpy(), rec["out"])


def test_c_oracle_on_golden_block(golden_dir):
    """The C restatement reproduces the layer-0 aggregation of the golden block."""
    rec = _load(golden_dir, "sage_mean_block")
    x, ei = rec["x"], rec["edge_index"]
    got = c_agg.agg_fwd(x, ei, x.shape[0], "mean")
    want = pyg_ref.propagate(torch.from_numpy(x), torch.from_numpy(ei), "mean").numpy()
    assert np.array_equal(got, want)


# ---- co-teaching loss restatement vs the reference's own CTLoss (fixtures)

@pytest.mark.parametrize("name", ["ct_loss_b300", "ct_loss_b1024"])
def test_ct_loss_oracle_matches_reference(golden_dir, name):
    from oracle import losses_ref
    g = np.load(os.path.join(golden_dir, name + ".npz"))
    y1 = torch.from_numpy(g["y1"]).requires_grad_(True)
    y2 = torch.from_numpy(g["y2"]).requires_grad_(True)
    out = losses_ref.ct_loss(y1, y2, torch.from_numpy(g["y_noise"]), float(g["forget_rate"]),
                             torch.from_numpy(g["ind"]), torch.from_numpy(g["noise_or_not"]))
    l1, l2, p1, p2, i1, i2, n1, n2 = out
    assert torch.equal(l1.detach(), torch.from_numpy(g["loss_1"]))
    assert torch.equal(l2.detach(), torch.from_numpy(g["loss_2"]))
    assert float(p1) == float(g["pure_ratio_1"]) and float(p2) == float(g["pure_ratio_2"])
    for got, key in ((i1, "ind_1_update"), (i2, "ind_2_update"), (n1, "ind_noisy_1"),
                     (n2, "ind_noisy_2")):
        assert np.array_equal(got.numpy(), g[key]), key
    l1.backward()
    l2.backward()
    assert torch.equal(y1.grad, torch.from_numpy(g["grad_y1"]))
    assert torch.equal(y2.grad, torch.from_numpy(g["grad_y2"]))
