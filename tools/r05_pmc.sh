#!/bin/bash
# Round-5 evidence: HBM traffic of the headline step's kernels (FETCH_SIZE and
# WRITE_SIZE in passes of their own, --kernel-trace only) and the Adam launch
# micro at three grid caps.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05pmc}; mkdir -p $O
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $c -d $O/pmc_$c -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-epoch --timer none > $O/pmc_$c.log 2>&1 || { tail -5 $O/pmc_$c.log; exit 1; }
done
echo pmc done
for w in 2 4 8; do
  NGNN_ADAM_WG_PER_CU=$w timeout -k 10 120 python3 tools/adam_micro.py > $O/adam_$w.log 2>&1 || exit 1
  echo "wg/cu $w: $(tail -1 $O/adam_$w.log)"
done
