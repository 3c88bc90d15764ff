#!/bin/bash
# A/B: kernel bench + step bench of earlier commits' worktrees under ab/ and HEAD.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-ab}; mkdir -p $O
for d in ${DIRS:-ab/*}; do
  n=$(basename $d)
  (cd $d && timeout -k 10 200 python3 tools/kbench_fwd.py) > $O/kbench_$n.json 2>&1 || exit $?
  (cd $d && timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-epoch) > $O/bench_$n.log 2>&1 || exit $?
done
timeout -k 10 200 python3 tools/kbench_fwd.py > $O/kbench_head.json 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-epoch --gather loader > $O/bench_head.log 2>&1 || exit $?
echo done
