#!/bin/bash
# Computers: the wide-path tests, then the bench at Adam's per-CU workgroup
# caps (NGNN_ADAM_WG_PER_CU) and the step breakdown at the best
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06awg}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  tail -1 $O/$n.log | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
}
A="--dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max"
step pytest 500 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_configs.py tests/test_optim_gpu.py -q -x --timeout 200 --timeout-method thread
for w in 2 4 3 8 2 4; do
  NGNN_ADAM_WG_PER_CU=$w step bench_w$w 300 python3 bench.py --no-cpu-baseline --no-eager-ref --no-epoch $A
done
echo done
