#!/bin/bash
# Round 6: fwd2 micro (main + fused stages) for each library in LIBS ("tree" =
# the in-tree build, else ablib/libngnn_NAME.so), interleaved twice
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r06lab}; mkdir -p $O
for pass in 1 2; do
for v in $LIBS; do
  if [ $v = tree ]; then L=""; else L=$PWD/ablib/libngnn_$v.so; fi
  NGNN_LIB=$L timeout -k 10 200 python tools/fwd2_micro.py --stages ${STAGES:-main,fused} --reps 50 > $O/micro_${v}_$pass.log 2>&1 || exit 3
  echo "$pass $v $(grep -E '^(main|fused|edge|narrow) ' $O/micro_${v}_$pass.log | tr -s ' ' | cut -d' ' -f1,2 | tr '\n' ' ')" | tee -a $O/summary.txt
done
done
