"""Where a kernel's spills (scratch_*) sit relative to its MFMAs / branches.
usage: python tools/asm_spills.py file.s <mangled-substring>"""
import re
import sys

s = open(sys.argv[1]).read()
key = sys.argv[2]
for m in re.finditer(r"^(_Z\S+):\s*;", s, re.M):
    name = m.group(1)
    if key not in name:
        continue
    end = s.find(".Lfunc_end", m.end())
    body = s[m.end():end].split("\n")
    marks = []
    for i, l in enumerate(body):
        t = l.strip()
        if t.startswith("scratch_"):
            marks.append((i, "S" + ("st" if "store" in t else "ld")))
        elif t.startswith("v_mfma"):
            marks.append((i, "M"))
        elif re.match(r"^\.LBB", t):
            marks.append((i, "L:" + t.split(":")[0]))
        elif t.startswith("s_cbranch") or t.startswith("s_branch"):
            marks.append((i, "B"))
    out, prev = [], None
    for i, k in marks:  # compress runs of MFMAs
        if k == "M" and prev == "M":
            out[-1] = (out[-1][0], "M", out[-1][2] + 1)
        else:
            out.append((i, k, 1))
        prev = k
    print(name, len(body), "lines,", sum(1 for _, k in marks if k.startswith("S")), "scratch ops")
    print(" ".join(f"{i}:{k}{'x%d' % n if n > 1 else ''}" for i, k, n in out))
