#!/bin/bash
# A/B of libngnn builds under ablib/ (NGNN_LIB) against the in-tree build:
# forward kernel bench + 1-GPU step bench each.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-abl}; mkdir -p $O
for v in head ${VARIANTS:-}; do
  if [ $v = head ]; then unset NGNN_LIB; else export NGNN_LIB=$PWD/ablib/$v.so; fi
  timeout -k 10 200 python3 tools/kbench_fwd.py > $O/kbench_$v.json 2>&1 || exit $?
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-epoch --gather ${GATHER:-loader} > $O/bench_$v.log 2>&1 || exit $?
done
echo done
