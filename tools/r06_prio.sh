#!/bin/bash
# epoch A/B: the sampling stream at normal vs high priority (NGNN_SIDE_PRIORITY)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06prio}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  python3 -c "import json,sys; d=json.loads(open('$O/$n.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('epoch_time_s'), d.get('epoch_time_s_sync_free_row_copy'), d.get('epoch_time_s_sync_loader'))"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
for p in 0 -1 0 -1; do
  NGNN_SIDE_PRIORITY=$p step bench_p$p 400 python3 bench.py --no-cpu-baseline --no-eager-ref
done
echo done
