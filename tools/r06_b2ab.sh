#!/bin/bash
# k_bwd2 A/B: the product library (this tree) against the profiling build
# in dbgb/ (an older k_bwd2, DBG=0): micro timings and rocprof kernel stats,
# then the bwd2 tests, the headline bench and its step breakdown
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06b2ab}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  tail -2 $O/$n.log | cut -c1-250
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step micro_new 120 python3 tools/bwd2_micro.py 100
NGNN_LIB=$PWD/dbgb/libngnn_dbg.so step micro_old 120 python3 tools/bwd2_micro.py 100
step micro_new2 120 python3 tools/bwd2_micro.py 100
step prof_new 200 rocprofv3 --kernel-trace --stats -d $O/prof_new -o run --output-format csv -- python3 tools/bwd2_micro.py 50
grep -h "k_bwd2" $O/prof_new/run_kernel_stats.csv | cut -c1-160
export NGNN_LIB=$PWD/dbgb/libngnn_dbg.so
step prof_old 200 rocprofv3 --kernel-trace --stats -d $O/prof_old -o run --output-format csv -- python3 tools/bwd2_micro.py 50
grep -h "k_bwd2" $O/prof_old/run_kernel_stats.csv | cut -c1-160
unset NGNN_LIB
step pytest 300 python -u -m pytest tests/test_gpu_bwd2.py tests/test_gpu_fold.py -q -x --timeout 120 --timeout-method thread
step bench_headline 400 python3 bench.py --no-cpu-baseline --no-eager-ref
step prof_headline 400 rocprofv3 --kernel-trace --stats -d $O/prof_headline -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --no-eager-ref --timer none
python3 tools/trace_step.py $O/prof_headline/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step_headline.txt 2>&1
cat $O/step_headline.txt
echo done
