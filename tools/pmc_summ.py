"""Average each PMC counter per dispatch over rocprofv3 counter-collection CSVs.

    python tools/pmc_summ.py gpurun_out/TAG [kernel-substring]
"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if sub not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("ngnn::", "")
        k = (name[-42:], r["Counter_Name"])
        agg[k] += float(r["Counter_Value"])
        disp[k].add((f, r["Dispatch_Id"]))
for k in sorted(agg):
    print(f"{k[0]:42s} {k[1]:32s} {agg[k] / len(disp[k]):16.1f}  (n={len(disp[k])})")
