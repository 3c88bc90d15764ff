#!/bin/bash
# HBM traffic of k_fwd2x / k_narrow_agg on the headline block (separate
# FETCH_SIZE and WRITE_SIZE passes, --kernel-trace only) for
# tools/pmc_traffic.py -> profiles/pmc_traffic.json
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r06pt}; mkdir -p $O
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "k_fwd2x|k_narrow_agg" -d $O/pmc_$c -o run --output-format csv -- python3 tools/fwd2_micro.py --stages fused,narrow --head --reps 10 > $O/pmc_$c.log 2>&1 || { tail -5 $O/pmc_$c.log; exit 1; }
done
echo traffic done
