"""Where the step period's idle time sits (run under rocprofv3 --kernel-trace):
the headline GraphedTrainStep driven three ways over the same pre-sampled
batches, phases separated by a device sync and marked by a 1-element fill:

  A  step(b) -- eager slot load + one graph replay (the bench loop)
  B  replay only, same loaded batch (graph after graph)
  C  load only (eager slot load after eager slot load)

    rocprofv3 --kernel-trace -d gpurun_out/gap -o run --output-format csv -- python3 tools/gap_micro.py
    python3 tools/gap_micro.py --report gpurun_out/gap/run_kernel_trace.csv
"""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "noise-gnn_amd"))


def _short(name):
    import re
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name[:28]


def report(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # the last four non-ngnn kernels are the phase marks (fills)
    marks = [i for i, r in enumerate(rows) if "ngnn" not in r["Kernel_Name"]][-4:]
    gaps = {}
    for ph, (i0, i1) in zip("ABC", zip(marks, marks[1:])):
        for k in range(i0 + 2, i1):
            prev, r = rows[k - 1], rows[k]
            g = (int(r["Start_Timestamp"]) - int(prev["End_Timestamp"])) / 1e3
            key = (ph, _short(prev["Kernel_Name"]), _short(r["Kernel_Name"]))
            gaps.setdefault(key, []).append(g)
    for (ph, a, b), v in sorted(gaps.items()):
        v.sort()
        print(f"{ph}  {a:28s} -> {b:28s} n={len(v):4d} median gap {v[len(v) // 2]:7.2f} us")


def main():
    import torch

    import ngnn
    from ngnn.graphs import GraphedTrainStep, slot_size
    from ngnn.loader import NeighborLoader, synthetic_graph
    from ngnn.optim import Adam

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    graph = synthetic_graph("ogbn-products", dev, seed=0)
    torch.manual_seed(1234)
    model = ngnn.SAGE(100, 256, 47, 2, dropout=0.5).to(dev)
    opt = Adam(model.parameters(), lr=1e-3)
    model.train()
    loader = NeighborLoader(graph, graph.train_idx, [15, 10], 1024, shuffle=True, seed=7)
    it = iter(loader)
    batches = [next(it) for _ in range(24)]
    n_cap, e_cap = slot_size(1024, [15, 10])
    gs = GraphedTrainStep(model, opt, 1024, n_cap, e_cap, batches[0].x.size(1), dev)
    gs.capture(batches[0].x, batches[0].edge_index, batches[0].y)
    for b in batches[:4]:
        gs(b.x, b.edge_index, b.y, b.batch_size)
    mark = torch.zeros(1, device=dev)
    torch.cuda.synchronize()
    mark.fill_(1.0)  # phase A
    for b in batches[4:24]:
        gs(b.x, b.edge_index, b.y, b.batch_size)
    torch.cuda.synchronize()
    mark.fill_(2.0)  # phase B
    b = batches[0]
    gs.load(b.x, b.edge_index, b.y, zero_copy=gs.zero_copy, batch_size=b.batch_size)
    for _ in range(20):
        gs.g_fb.replay()
    torch.cuda.synchronize()
    mark.fill_(3.0)  # phase C
    for b in batches[4:24]:
        gs.load(b.x, b.edge_index, b.y, zero_copy=gs.zero_copy, batch_size=b.batch_size)
    torch.cuda.synchronize()
    mark.fill_(4.0)
    torch.cuda.synchronize()
    print("gap_micro done")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--report":
        report(sys.argv[2])
    else:
        main()
