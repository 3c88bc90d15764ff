"""Generate the golden fixtures in tests/golden/*.npz.

Run in the build container (the reference checkout is only present there):

    python tests/golden/make_golden.py  [--ref /root/reference]

How the vectors are made: the reference's OWN model files
``src/models/layers/sage.py`` and ``src/models/layers/convolution.py`` are
imported from the read-only checkout and executed.  Their only missing
dependency, ``torch_geometric.nn`` (PyG 2.5.1, un-vendored, not installable
offline), is supplied by ``oracle.pyg_ref`` (torch-CPU restatement of the PyG
op sequence).  So the fixtures pin the reference's wrapper composition
(layer loop, relu/dropout/bn placement, last-layer logits, layer-wise
``inference``) and its state-dict contract; the conv arithmetic is pinned by
the hand-computed known-answer tests in tests/test_oracle.py.

Only tensors are written (inputs, weights, outputs, gradients); no reference
source or bytecode is stored.  Every case records its seed.
"""
from __future__ import annotations

import argparse
import functools
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import pyg_ref  # noqa: E402


def install_shim(default_aggr: str = "mean"):
    pyg = types.ModuleType("torch_geometric")
    pyg_nn = types.ModuleType("torch_geometric.nn")
    pyg_nn.SAGEConv = functools.partial(pyg_ref.SAGEConv, aggr=default_aggr)
    pyg_nn.GCNConv = pyg_ref.GCNConv
    pyg_nn.global_mean_pool = lambda *a, **k: None  # imported, unused (convolution.py:5)
    pyg.nn = pyg_nn
    sys.modules["torch_geometric"] = pyg
    sys.modules["torch_geometric.nn"] = pyg_nn


def import_reference(ref: str, default_aggr: str = "mean"):
    install_shim(default_aggr)
    if ref not in sys.path:
        sys.path.insert(0, ref)
    for m in ["src.models.layers.sage", "src.models.layers.convolution"]:
        sys.modules.pop(m, None)
    import importlib
    sage = importlib.import_module("src.models.layers.sage")
    conv = importlib.import_module("src.models.layers.convolution")
    return sage, conv


def block_graph(seed: int, n_seeds: int, fanouts, n_graph: int):
    """NeighborLoader-like sampled block: seeds first, dst-sorted local edges.

    Mirrors the layout PyG's NeighborLoader hands to pipeline.py:155: node ids
    are local, n_id starts with the seeds, hop-k nodes follow hop-(k-1) nodes,
    edges are grouped by destination in frontier order (row 0 = source).
    """
    g = torch.Generator().manual_seed(seed)
    deg = torch.randint(0, 12, (n_graph,), generator=g)
    nbrs = [torch.randint(0, n_graph, (int(d),), generator=g) for d in deg]
    seeds = torch.randperm(n_graph, generator=g)[:n_seeds]
    n_id = list(seeds.tolist())
    local = {v: i for i, v in enumerate(n_id)}
    frontier = list(range(len(n_id)))
    src, dst = [], []
    for k in fanouts:
        nxt = []
        for li in frontier:
            v = n_id[li]
            cand = nbrs[v]
            if len(cand) > k:
                cand = cand[torch.randperm(len(cand), generator=g)[:k]]
            for u in cand.tolist():
                if u not in local:
                    local[u] = len(n_id)
                    n_id.append(u)
                    nxt.append(local[u])
                src.append(local[u])
                dst.append(li)
        frontier = nxt
    ei = torch.tensor([src, dst], dtype=torch.long).reshape(2, -1)
    return torch.tensor(n_id), ei


def random_graph(seed: int, n: int, e: int, sort_by: str | None):
    g = torch.Generator().manual_seed(seed)
    ei = torch.randint(0, n, (2, e), generator=g)
    if sort_by == "dst":
        ei = ei[:, torch.argsort(ei[1], stable=True)]
    elif sort_by == "src":
        ei = ei[:, torch.argsort(ei[0], stable=True)]
    return ei


def run_model_case(model, x, ei, seed, train=False):
    model.train(train)
    xr = x.clone().requires_grad_(True)
    torch.manual_seed(seed + 7)
    out = model(xr, ei)
    gseed = torch.Generator().manual_seed(seed + 11)
    G = torch.randn(out.shape, generator=gseed)
    (out * G).sum().backward()
    rec = {"x": x.numpy(), "edge_index": ei.numpy(), "out": out.detach().numpy(),
           "grad_out": G.numpy(), "grad_x": xr.grad.numpy()}
    for k, v in model.state_dict().items():
        rec["param/" + k] = v.detach().numpy().copy()
    for k, p in model.named_parameters():
        rec["grad/" + k] = p.grad.detach().numpy().copy()
    return rec


def ct_loss_cases(ref: str):
    if ref not in sys.path:
        sys.path.insert(0, ref)
    import importlib
    losses = importlib.import_module("src.utils.losses")
    out = {}
    for name, B, C, n_graph, forget, seed in [("ct_loss_b300", 300, 47, 1000, 0.2, 1000),
                                              ("ct_loss_b1024", 1024, 40, 5000, 0.45, 1001)]:
        g = torch.Generator().manual_seed(seed)
        y1 = (2 * torch.randn(B, C, generator=g)).requires_grad_(True)
        y2 = (2 * torch.randn(B, C, generator=g)).requires_grad_(True)
        yn = torch.randint(0, C, (B,), generator=g)
        ind = torch.randperm(n_graph, generator=g)[:B]
        clean = torch.rand(n_graph, generator=g) < 0.7
        crit = losses.CTLoss("cpu")
        l1, l2, p1, p2, i1, i2, n1, n2 = crit(y1, y2, yn, forget, ind, clean)
        l1.backward()
        l2.backward()
        out[name] = {"y1": y1.detach().numpy(), "y2": y2.detach().numpy(), "y_noise": yn.numpy(),
                     "ind": ind.numpy(), "noise_or_not": clean.numpy(),
                     "forget_rate": np.array(forget), "loss_1": l1.detach().numpy(),
                     "loss_2": l2.detach().numpy(), "pure_ratio_1": np.asarray(p1, dtype=np.float32),
                     "pure_ratio_2": np.asarray(p2, dtype=np.float32),
                     "ind_1_update": np.asarray(i1), "ind_2_update": np.asarray(i2),
                     "ind_noisy_1": np.asarray(n1), "ind_noisy_2": np.asarray(n2),
                     "grad_y1": y1.grad.numpy(), "grad_y2": y2.grad.numpy(), "meta/seed": np.array(seed)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default=None, help="comma list of case names to (re)write")
    args = ap.parse_args()
    out_dir = HERE
    cases = {}

    sage_m, conv_m = import_reference(args.ref, "mean")

    # 1. products-like block, mean, 2 layers (100 -> 32 -> 47), eval mode
    torch.manual_seed(100)
    n_id, ei = block_graph(1, 12, [15, 10], 250)
    x = torch.randn(len(n_id), 100, generator=torch.Generator().manual_seed(2))
    m = sage_m.SAGE(100, 32, 47, 2, dropout=0.5)
    cases["sage_mean_block"] = run_model_case(m, x, ei, 100)
    cases["sage_mean_block"]["meta/batch_size"] = np.array(12)

    # 2. 3-layer mean, unsorted random edges, duplicates + self loops possible
    torch.manual_seed(200)
    ei = random_graph(3, 90, 700, None)
    x = torch.randn(90, 24, generator=torch.Generator().manual_seed(4))
    m = sage_m.SAGE(24, 40, 7, 3, dropout=0.5)
    cases["sage_mean_3layer_unsorted"] = run_model_case(m, x, ei, 200)

    # 3. src-sorted edges (augmentation.py:82-85 order), width 128 (arxiv-like)
    torch.manual_seed(300)
    ei = random_graph(5, 70, 500, "src")
    x = torch.randn(70, 128, generator=torch.Generator().manual_seed(6))
    m = sage_m.SAGE(128, 64, 40, 2, dropout=0.5)
    cases["sage_mean_srcsorted"] = run_model_case(m, x, ei, 300)

    # 4. use_bn=True, dropout=0, train mode (batch statistics)
    torch.manual_seed(400)
    ei = random_graph(7, 60, 300, "dst")
    x = torch.randn(60, 16, generator=torch.Generator().manual_seed(8))
    m = sage_m.SAGE(16, 32, 5, 2, dropout=0.0, use_bn=True)
    cases["sage_mean_bn_train"] = run_model_case(m, x, ei, 400, train=True)

    # 5. SimpleGCN (GCNConv normalize=False), 2 and 3 layers
    torch.manual_seed(500)
    ei = random_graph(9, 80, 600, "dst")
    x = torch.randn(80, 20, generator=torch.Generator().manual_seed(10))
    m = conv_m.SimpleGCN(20, 32, 6, 2, dropout=0.5)
    cases["gcn_2layer"] = run_model_case(m, x, ei, 500)
    torch.manual_seed(600)
    ei = random_graph(11, 50, 400, None)
    x = torch.randn(50, 12, generator=torch.Generator().manual_seed(12))
    m = conv_m.SimpleGCN(12, 16, 16, 3, dropout=0.5)
    cases["gcn_3layer_unsorted"] = run_model_case(m, x, ei, 600)

    # 6. max aggregation (config_amazon-like input width, 767 -> 16 -> 10); the
    #    reference never sets aggr, so the shim's SAGEConv default is 'max' here.
    sage_x, _ = import_reference(args.ref, "max")
    torch.manual_seed(700)
    n_id, ei = block_graph(13, 6, [10, 5], 40)
    x = torch.randn(len(n_id), 767, generator=torch.Generator().manual_seed(14))
    m = sage_x.SAGE(767, 16, 10, 2, dropout=0.5)
    cases["sage_max_block"] = run_model_case(m, x, ei, 700)
    # max with ties (relu'd, rounded features): exercises the tie-split rule
    torch.manual_seed(800)
    ei = random_graph(15, 40, 300, "dst")
    x = torch.relu(torch.randn(40, 8, generator=torch.Generator().manual_seed(16))).round()
    m = sage_x.SAGE(8, 8, 3, 2, dropout=0.5)
    cases["sage_max_ties"] = run_model_case(m, x, ei, 800)

    # 7. layer-wise inference (sage.py:42-58) over a fake subgraph loader
    sage_m, _ = import_reference(args.ref, "mean")
    torch.manual_seed(900)
    n_graph = 48
    gg = torch.Generator().manual_seed(17)
    x_all = torch.randn(n_graph, 10, generator=gg)
    m = sage_m.SAGE(10, 12, 4, 2, dropout=0.5).eval()
    batches = []
    for b, seeds in enumerate([torch.arange(0, 24), torch.arange(24, 48)]):
        n_id, ei = block_graph(30 + b, 24, [4, 3], n_graph)
        # replace seeds with the loader's contiguous input_nodes=None order
        perm = {int(v): i for i, v in enumerate(n_id.tolist())}
        order = seeds.tolist() + [v for v in n_id.tolist() if v not in set(seeds.tolist())]
        remap = torch.tensor([order.index(v) for v in n_id.tolist()])
        batches.append(types.SimpleNamespace(n_id=torch.tensor(order), edge_index=remap[ei],
                                             batch_size=24))
        del perm
    with torch.no_grad():
        inf = m.inference(x_all, batches, "cpu")
    rec = {"x_all": x_all.numpy(), "out": inf.numpy()}
    for i, bt in enumerate(batches):
        rec[f"batch{i}/n_id"] = bt.n_id.numpy()
        rec[f"batch{i}/edge_index"] = bt.edge_index.numpy()
        rec[f"batch{i}/batch_size"] = np.array(bt.batch_size)
    for k, v in m.state_dict().items():
        rec["param/" + k] = v.numpy().copy()
    cases["sage_inference"] = rec

    # 8. co-teaching loss (src/utils/losses.py:19-49, imported from the checkout):
    #    tie-free continuous logits; forward outputs, kept indices, and the
    #    gradients of each model's loss
    cases.update(ct_loss_cases(args.ref))

    if args.only:
        keep = set(args.only.split(","))
        cases = {k: v for k, v in cases.items() if k in keep}
    total = 0
    for name, rec in cases.items():
        path = os.path.join(out_dir, name + ".npz")
        np.savez_compressed(path, **rec)
        total += os.path.getsize(path)
        print(f"{name}: {os.path.getsize(path) / 1024:.1f} KiB, keys={len(rec)}")
    print(f"total {total / 1024:.1f} KiB")


if __name__ == "__main__":
    main()
