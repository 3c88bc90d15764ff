#!/bin/bash
# Round 6: smoke(), and the data-parallel bench path rehearsed on two gloo
# ranks on the one GPU WITH its epochs (the sync-free loader under DP)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06run6}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
tail -1 $O/smoke.log
NGNN_DIST_BACKEND=gloo step dp2_headline 600 python3 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-eager-ref
tail -1 $O/dp2_headline.log | cut -c1-400
NGNN_DIST_BACKEND=gloo step dp2_coteaching 600 python3 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-eager-ref --coteaching
tail -1 $O/dp2_coteaching.log | cut -c1-300
echo done
