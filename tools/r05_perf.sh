#!/bin/bash
# per-launch micro + headline bench for each library in LIBS ("tree" = in-tree build)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05pf}; mkdir -p $O
for v in $LIBS; do
  if [ $v = tree ]; then L=""; else L=$PWD/ablib/libngnn_$v.so; fi
  NGNN_LIB=$L timeout -k 10 300 python tools/fwd2_micro.py --stages ${STAGES:-main} --reps 50 > $O/micro_$v.log 2>&1 || exit 3
  NGNN_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-epoch --no-eager-ref > $O/bench_$v.log 2>&1 || exit 4
  echo "$v $(grep -E '^(main|edge|narrow)' $O/micro_$v.log | tr -s ' ' | tr '\n' ' ') step $(tail -n1 $O/bench_$v.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" | tee -a $O/summary.txt
done
