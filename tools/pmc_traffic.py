"""HBM traffic per launch from separate FETCH_SIZE / WRITE_SIZE rocprofv3
passes (tools/gpu_pmc.sh), mapped to bench.py's timer spans, written to
profiles/pmc_traffic.json (read by bench.py for roofline.traffic), keyed
"span|workload|dtype" so a line only ever carries its own workload's traffic.

FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the
bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM section), so it is
doubled; WRITE_SIZE is exact for 16-B stores.

    python tools/pmc_traffic.py gpurun_out/TAG --map sage_fwd_l0='k_sage_rt<16,' \
        --map sage_fwd_l1='k_sage_rt<3,' [--out profiles/pmc_traffic.json]
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--map", action="append", default=[], help="span=kernel-name-substring")
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    ap.add_argument("--workload", default="products-[15,10]-bs1024",
                    help="bench.py config.workload the profiled command ran")
    ap.add_argument("--dtype", default="f32")
    a = ap.parse_args()
    # span=substring[@k/m]: of the matching dispatches (in dispatch order),
    # the k-th of every m (a kernel that runs for several layers of a step)
    spans, nth = {}, {}
    for m in a.map:
        span, sub = m.split("=", 1)
        if "@" in sub:
            sub, km = sub.rsplit("@", 1)
            nth[span] = tuple(int(v) for v in km.split("/"))
        spans[span] = sub
    # (span, counter) -> {dispatch: summed value}
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for f in sorted(glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace(" ", "")
            for span, sub in spans.items():
                if sub.replace(" ", "") in k:
                    acc[(span, r["Counter_Name"])][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
                    names[span] = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    out = {}
    if os.path.exists(a.out):
        out = json.load(open(a.out))
    def pick(span, counter):
        d = acc[(span, counter)]
        if span not in nth:
            return list(d.values())
        k, m = nth[span]
        keys = sorted(d, key=lambda fd: (fd[0], int(fd[1])))
        return [d[fd] for i, fd in enumerate(keys) if i % m == k]

    for span in spans:
        fv = pick(span, "FETCH_SIZE")
        wv = pick(span, "WRITE_SIZE")
        if not fv or not wv:
            print(f"{span}: no FETCH_SIZE/WRITE_SIZE rows")
            continue
        fetch = 2 * 1024 * statistics.mean(fv)
        write = 1024 * statistics.mean(wv)
        out[f"{span}|{a.workload}|{a.dtype}"] = {"kernel": names[span], "fetch_bytes": int(fetch), "write_bytes": int(write),
                     "traffic_bytes": int(fetch + write), "dispatches": [len(fv), len(wv)],
                     "source": os.path.basename(os.path.normpath(a.dir))}
        print(span, out[f"{span}|{a.workload}|{a.dtype}"])
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
