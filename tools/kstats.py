"""Compact view of a rocprofv3 kernel_stats.csv: ngnn kernels by name +
template arguments, then the top others.  usage: kstats.py DIR_OR_CSV [steps]"""
import csv, glob, os, re, sys

p = sys.argv[1]
f = p if p.endswith(".csv") else glob.glob(os.path.join(p, "**", "*kernel_stats.csv"), recursive=True)[0]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 0
pat = re.compile(r"ngnn::(?:\(anonymous namespace\)::)?(\w+(?:<[^()]*>)?)")
ours, other = [], []
for r in csv.DictReader(open(f)):
    m = pat.search(r["Name"])
    rec = (int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e3,
           m.group(1) if m else r["Name"][:90])
    (ours if m else other).append(rec)
for title, lst in (("ngnn", ours), ("other (top 12)", other[:12])):
    print(f"-- {title}")
    for c, avg, tot, n in lst:
        per = f" {tot / steps:8.1f} us/step" if steps else ""
        print(f"{c:6d} {avg:9.1f} us{per}  {n}")
