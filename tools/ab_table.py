"""Side-by-side kbench / bench of an ab_libs.sh output directory."""
import glob
import json
import os
import sys

d = sys.argv[1]
ks = {}
for f in sorted(glob.glob(d + "/kbench_*.json")):
    t = open(f).read()
    ks[os.path.basename(f)[7:-5]] = json.loads(t[t.index("{"):])
for n in ks:
    for line in open(f"{d}/bench_{n}.log"):
        if line.startswith("{"):
            r = json.loads(line)
            print(n, r["ms_per_step"], {k: v["avg_us"] for k, v in r["roofline"]["all_kernels"].items()})
keys = sorted(set().union(*[k.keys() for k in ks.values()]))
print(" " * 24, " ".join(f"{n:>9s}" for n in ks))
for k in keys:
    print(f"{k:24s}", " ".join(f"{str(ks[n].get(k, '-')):>9s}" for n in ks))
