#!/bin/bash
# k_fwd2x store policy per output, in the step: tree (h / z / out
# non-temporal) against abv/ variants (all cached; z, z+out, h cached):
# bench ms/step interleaved twice, then rocprof breakdowns of tree and the
# variants
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06sa}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for pass in 1 2; do
  for v in ${VARS:-tree all0 z0 zo0 h0}; do
    if [ $v = tree ]; then L=""; else L=$PWD/abv/libngnn_$v.so; fi
    NGNN_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eager-ref --no-epoch > $O/bench_${v}_$pass.log 2>&1 || exit 3
    echo "$pass $v $(tail -1 $O/bench_${v}_$pass.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" | tee -a $O/summary.txt
  done
done
for v in ${PVARS:-tree all0 z0}; do
  if [ $v = tree ]; then L=""; else L=$PWD/abv/libngnn_$v.so; fi
  NGNN_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --no-eager-ref --timer none > $O/prof_$v.log 2>&1 || exit 3
  python3 tools/trace_step.py $O/prof_$v/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step_$v.txt 2>&1
  echo "== $v" | tee -a $O/summary.txt; head -8 $O/step_$v.txt | tee -a $O/summary.txt
done
echo done
