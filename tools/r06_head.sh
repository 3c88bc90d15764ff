#!/bin/bash
# loss head: group tickets a line apart -- head / graph / co-teaching tests,
# headline bench + step breakdown
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06hd}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  tail -1 $O/$n.log | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step pytest 600 python -u -m pytest tests/test_gpu_head.py tests/test_graphs_gpu.py tests/test_coteaching_gpu.py tests/test_gpu_bwd2.py tests/test_losses_gpu.py tests/test_gpu_configs.py -q -x --timeout 200 --timeout-method thread
step bench_headline 400 python3 bench.py --no-cpu-baseline --no-eager-ref
step prof_headline 400 rocprofv3 --kernel-trace --stats -d $O/prof_headline -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --no-eager-ref --timer none
python3 tools/trace_step.py $O/prof_headline/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step_headline.txt 2>&1
cat $O/step_headline.txt
A="--dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max"
step bench_c 300 python3 bench.py --no-cpu-baseline --no-eager-ref --no-epoch $A
step prof_c 300 rocprofv3 --kernel-trace --stats -d $O/prof_c -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --no-eager-ref --timer none $A
python3 tools/trace_step.py $O/prof_c/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step_c.txt 2>&1
cat $O/step_c.txt
echo done
