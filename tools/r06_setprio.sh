#!/bin/bash
# static priority for waves 4-7 (abv/ variants) against the tree: k_fwd2x and
# k_bwd2 micros interleaved, then the headline bench per library
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06sp}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for pass in 1 2; do
  for v in tree f2prio; do
    if [ $v = tree ]; then L=""; else L=$PWD/abv/libngnn_$v.so; fi
    NGNN_LIB=$L timeout -k 10 200 python3 tools/fwd2_micro.py --stages fused --reps 50 > $O/f2_${v}_$pass.log 2>&1 || exit 3
    echo "$pass $v $(grep -E '^fused ' $O/f2_${v}_$pass.log | tr -s ' ' | cut -d' ' -f1,2)" | tee -a $O/summary.txt
  done
  for v in tree b2prio; do
    if [ $v = tree ]; then L=""; else L=$PWD/abv/libngnn_$v.so; fi
    NGNN_LIB=$L timeout -k 10 200 python3 tools/bwd2_micro.py 100 > $O/b2_${v}_$pass.log 2>&1 || exit 3
    echo "$pass $v $(grep us/call $O/b2_${v}_$pass.log)" | tee -a $O/summary.txt
  done
done
for v in tree f2prio b2prio tree; do
  if [ $v = tree ]; then L=""; else L=$PWD/abv/libngnn_$v.so; fi
  NGNN_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eager-ref --no-epoch > $O/bench_$v.log 2>&1 || exit 3
  echo "bench $v $(tail -1 $O/bench_$v.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" | tee -a $O/summary.txt
done
echo done
