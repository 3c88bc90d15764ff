#!/bin/bash
# Forward-kernel phase ablation (NGNN_SAGE_ABLATE bits, row-tile kernel: 1 no
# MFMA, 2 no output stores, 4 no x loads).  One process per mode.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-ablate}; mkdir -p "$OUT"
for m in ${MODES:-0 1 2 4 3 5 6 7}; do
  NGNN_SAGE_ABLATE=$m timeout -k 10 200 python3 tools/bench_kernels.py --reps 10 > "$OUT/mode$m.json" 2> "$OUT/mode$m.err"
  rc=$?; echo "mode $m rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
echo done
