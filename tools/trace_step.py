"""Per-step kernel breakdown from a rocprofv3 --kernel-trace CSV.

Finds the steady-state training steps (delimited by launches whose name
contains --marker, default the first fused layer kernel) and prints the
median duration of every kernel slot of a step plus the step's wall span.

    python tools/trace_step.py gpurun_out/TAG/prof/run_kernel_trace.csv
"""
import argparse
import collections
import csv
import statistics


def short(name, n=90):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return name[:n]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="k_sage_fwd<4, 4")
    ap.add_argument("--skip", type=int, default=3, help="steps to skip (warmup)")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(idx) < a.skip + 2:
        print("not enough marker launches", len(idx))
        return
    steps = []
    for s in range(a.skip, min(len(idx) - 1, a.skip + a.steps)):
        steps.append(rows[idx[s]:idx[s + 1]])
    per = collections.defaultdict(list)
    spans, busy = [], []
    for st in steps:
        t0 = int(st[0]["Start_Timestamp"])
        t1 = int(st[-1]["End_Timestamp"])
        spans.append((t1 - t0) / 1e3)
        b = 0
        for j, r in enumerate(st):
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            per[(j, short(r["Kernel_Name"]))].append(d)
            b += d
        busy.append(b)
    print(f"steps analysed: {len(steps)}  kernels/step: {len(steps[0])}")
    print(f"step span (first launch -> last end): median {statistics.median(spans):.1f} us; "
          f"sum of kernel times: median {statistics.median(busy):.1f} us")
    tot = statistics.median(busy)
    for (j, n), ds in sorted(per.items()):
        m = statistics.median(ds)
        print(f"  {j:3d} {m:8.1f} us {100 * m / tot:5.1f}%  {n}")


if __name__ == "__main__":
    main()
