#!/bin/bash
# ABI 21: the Adam ticket's group words a line apart -- micro, tests, Computers
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06at}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  tail -1 $O/$n.log | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step pytest 500 python -u -m pytest tests/test_optim_gpu.py tests/test_gpu_fold.py tests/test_graphs_gpu.py -q -x --timeout 200 --timeout-method thread
step micro 120 python3 tools/adam_micro.py
step prof 120 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/adam_micro.py
python3 -c "
import csv
for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    if 'adam' in r['Name']: print('   ', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')"
NGNN_ADAM_WG_PER_CU=1 step micro_w1 120 python3 tools/adam_micro.py
A="--dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max"
step bench_c1 300 python3 bench.py --no-cpu-baseline --no-eager-ref --no-epoch $A
step bench_c2 300 python3 bench.py --no-cpu-baseline --no-eager-ref --no-epoch $A
echo done
