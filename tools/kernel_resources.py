"""Print VGPR / spill / occupancy per kernel from hipcc -Rpass-analysis output.
usage: python tools/kernel_resources.py noise-gnn_amd/csrc/ngnn_sage.hip [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
       "-Iinclude", "-Inoise-gnn_amd/csrc", "-c", src, "-o", "/dev/null",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = {}
rows = []
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?): (.*?) \[", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        if cur:
            rows.append(cur)
        cur = {"name": v}
    else:
        cur[k] = v
if cur:
    rows.append(cur)
dem = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                     text=True).stdout.splitlines()
for r, d in zip(rows, dem):
    if flt in d:
        d = re.sub(r"\(.*", "", d.replace("ngnn::(anonymous namespace)::", ""))
        print(f"{d:45s} VGPR {r.get('VGPRs','?'):>4} AGPR {r.get('AGPRs','?'):>3} spill {r.get('VGPRs Spill','?'):>3} "
              f"LDS {r.get('LDS Size [bytes/block]','?'):>6} occ {r.get('Occupancy [waves/SIMD]','?')}")
