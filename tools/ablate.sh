#!/bin/bash
# Forward-kernel phase ablation (NGNN_SAGE_ABLATE bits: 1 no MFMA, 2 no output
# stores, 4 no X staging, 8 no epilogue).  One process per mode.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-ablate}; mkdir -p "$OUT"
for m in ${MODES:-0 1 2 4 8 12 5 11}; do
  NGNN_SAGE_ABLATE=$m timeout -k 10 200 python3 tools/bench_kernels.py --reps 10 > "$OUT/mode$m.json" 2> "$OUT/mode$m.err"
  rc=$?; echo "mode $m rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
echo done
