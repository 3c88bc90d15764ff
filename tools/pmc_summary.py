"""Summarise rocprofv3 --pmc passes: per kernel (name filter), the mean over
dispatches of each counter summed over its per-instance rows.
    python tools/pmc_summary.py gpurun_out/TAG [--filter k_sage_rt]"""
import argparse
import collections
import csv
import glob
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--filter", default="k_sage_rt")
    a = ap.parse_args()
    # (kernel, counter) -> {dispatch: value}
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if a.filter not in k:
                continue
            k = k.replace("void ", "").replace("(anonymous namespace)::", "").replace("ngnn::", "").split("(")[0]
            key = (f, r["Dispatch_Id"])
            acc[(k, r["Counter_Name"])][key] += float(r["Counter_Value"])
            dur[k][key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    kernels = sorted({k for k, _ in acc})
    for k in kernels:
        ds = list(dur[k].values())
        print(f"== {k}  dispatches {len(ds)}  median {statistics.median(ds):.1f} us")
        for (kk, c), vals in sorted(acc.items()):
            if kk == k:
                v = list(vals.values())
                print(f"   {c:32s} {statistics.mean(v):16.4g}")


if __name__ == "__main__":
    main()
