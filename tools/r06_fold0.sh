#!/bin/bash
# ABI 22: the input layer's Adam step in its weight-gradient reduction --
# fold / optimizer / config / graph tests, Computers bench + breakdown
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06f0}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  tail -1 $O/$n.log | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step pytest 700 python -u -m pytest tests/test_gpu_fold.py tests/test_optim_gpu.py tests/test_gpu_configs.py tests/test_graphs_gpu.py -q -x --timeout 250 --timeout-method thread
A="--dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max"
step bench_c1 300 python3 bench.py --no-cpu-baseline --no-eager-ref --no-epoch $A
step bench_c2 300 python3 bench.py --no-cpu-baseline --no-eager-ref --no-epoch $A
step prof_c 300 rocprofv3 --kernel-trace --stats -d $O/prof_c -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --no-eager-ref --timer none $A
python3 tools/trace_step.py $O/prof_c/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step_c.txt 2>&1
cat $O/step_c.txt
echo done
