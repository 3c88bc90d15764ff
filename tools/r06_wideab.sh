#!/bin/bash
# Computers A/B: the wide H2 preparation riding on the aggregate launch (this
# tree) against dbgb/ (the separate k_wide_prep_h2 launch); wide-path tests
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06wab}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  tail -1 $O/$n.log | cut -c1-330
  if [ $rc -ne 0 ]; then exit $rc; fi
}
A="--dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max"
step pytest 400 python -u -m pytest tests/test_gpu_configs.py -k computers tests/test_gpu_fused.py -q -x --timeout 120 --timeout-method thread
step bench_new 300 python3 bench.py --no-cpu-baseline --no-eager-ref --no-epoch $A
NGNN_LIB=$PWD/dbgb/libngnn_dbg.so step bench_old 300 python3 bench.py --no-cpu-baseline --no-eager-ref --no-epoch $A
step bench_new2 300 python3 bench.py --no-cpu-baseline --no-eager-ref --no-epoch $A
step prof_new 300 rocprofv3 --kernel-trace --stats -d $O/prof_new -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --no-eager-ref --timer none $A
python3 tools/trace_step.py $O/prof_new/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step_new.txt 2>&1
cat $O/step_new.txt
echo done
