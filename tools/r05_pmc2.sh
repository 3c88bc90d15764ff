#!/bin/bash
# HBM traffic per launch of the fused two-layer forward (k_fwd2x) and the
# head launch on the headline block (tools/fwd2_micro.py: R'-bounded h as in
# the step), FETCH_SIZE / WRITE_SIZE in passes of their own.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05pmc2}; mkdir -p $O
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "k_fwd2x|k_narrow_agg" -d $O/pmc_$c -o run --output-format csv -- python3 tools/fwd2_micro.py --stages fused,narrow --head --reps 10 > $O/pmc_$c.log 2>&1 || { tail -5 $O/pmc_$c.log; exit 1; }
done
timeout -k 10 120 python3 tools/fwd2_micro.py --stages fused,edge,main,narrow --head --reps 50 > $O/micro.log 2>&1 || exit 1
cat $O/micro.log | tail -6
