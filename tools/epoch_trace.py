"""Where an epoch's time goes, from a rocprofv3 --kernel-trace CSV of
bench.py (whose last phase is the epoch over the loader).

Takes the last --batches windows that start at a sampler launch (k_sb_init,
one per batch) and reports, per window and in total: wall time, the busy
time (union of kernel intervals, any stream), the sampler's kernels
(k_sb_*, k_gather_rows*), the training step's kernels, and the idle gap.

    python tools/epoch_trace.py gpurun_out/TAG/prof/run_kernel_trace.csv --batches 193
"""
import argparse
import collections
import csv
import statistics


def union_len(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--batches", type=int, default=193)
    ap.add_argument("--marker", default="k_sb_init")
    ap.add_argument("--skip-last", type=int, default=0,
                    help="windows to leave out at the end (bench.py's second, fused-gather epoch)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if a.skip_last:
        idx = idx[:-a.skip_last]
    idx = idx[-(a.batches + 1):]
    win = collections.defaultdict(list)
    names = collections.defaultdict(list)
    for w in range(len(idx) - 1):
        rs = rows[idx[w]:idx[w + 1]]
        t0 = int(rs[0]["Start_Timestamp"])
        t1 = int(rows[idx[w + 1]]["Start_Timestamp"])
        iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rs]
        samp = [(s, e) for (s, e), r in zip(iv, rs) if "k_sb_" in r["Kernel_Name"] or "k_gather_rows" in r["Kernel_Name"]]
        step = [(s, e) for (s, e), r in zip(iv, rs) if not ("k_sb_" in r["Kernel_Name"] or "k_gather_rows" in r["Kernel_Name"])]
        win["wall_us"].append((t1 - t0) / 1e3)
        win["busy_us"].append(union_len(iv) / 1e3)
        win["sampler_kernels_us"].append(sum(e - s for s, e in samp) / 1e3)
        win["sampler_span_us"].append((max(e for _, e in samp) - min(s for s, _ in samp)) / 1e3 if samp else 0.0)
        win["step_kernels_us"].append(sum(e - s for s, e in step) / 1e3)
        win["launches"].append(len(rs))
        for r in rs:
            n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
            names[n.split("(")[0][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    nb = len(win["wall_us"])
    print(f"batches analysed: {nb}")
    for k, v in win.items():
        print(f"  {k:22s} median {statistics.median(v):9.1f}   total {sum(v) / 1e3:9.2f} ms" if k != "launches"
              else f"  {k:22s} median {statistics.median(v):9.1f}")
    print("per-kernel (median us, launches per batch):")
    for n, ds in sorted(names.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {statistics.median(ds):8.1f} us  x{len(ds) / max(nb, 1):5.2f}  {n}")


if __name__ == "__main__":
    main()
