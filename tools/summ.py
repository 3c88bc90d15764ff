"""Summarise the bench JSON lines of a gpurun_out/<tag>/ directory."""
import glob
import json
import sys

for f in sorted(glob.glob(sys.argv[1] + "/bench*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            r = d["roofline"] or {}
            ks = " ".join(f"{k}:{v['avg_us']}" for k, v in r.get("all_kernels", {}).items())
            print(f"{f.split('/')[-1]:26s} {d['value'] / 1e6:8.1f}M {d['ms_per_step']:.4f}ms "
                  f"ep={d['epoch_time_s']} {d.get('feature_gather', '')[:5]} | {r.get('bound')} "
                  f"frac={r.get('frac')} | {ks}")
