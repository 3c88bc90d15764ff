#!/bin/bash
# slot load with one r_next atomic per workgroup; Adam loads a stride ahead:
# graph / loader / optimizer tests, headline bench + breakdown, Computers
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06slot}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  tail -1 $O/$n.log | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step pytest 600 python -u -m pytest tests/test_graphs_gpu.py tests/test_optim_gpu.py tests/test_gpu_fold.py tests/test_loader_gpu.py tests/test_gpu_head.py -q -x --timeout 200 --timeout-method thread
step bench_headline 400 python3 bench.py --no-cpu-baseline --no-eager-ref
step prof_headline 400 rocprofv3 --kernel-trace --stats -d $O/prof_headline -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --no-eager-ref --timer none
python3 tools/trace_step.py $O/prof_headline/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step_headline.txt 2>&1
cat $O/step_headline.txt
A="--dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max"
step bench_c 300 python3 bench.py --no-cpu-baseline --no-eager-ref --no-epoch $A
echo done
