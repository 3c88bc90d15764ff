#!/bin/bash
# rocprof kernel stats of the graph-replay bench, fused vs loader feature gather,
# plus kbench/bench of the ab/ worktrees listed in DIRS.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-pab}; mkdir -p $O
export TMPDIR=/tmp
for g in fused loader; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$g" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --timer none --gather $g > "$O/prof_$g.log" 2>&1 || exit $?
done
for d in ${DIRS:-}; do
  n=$(basename $d)
  (cd $d && timeout -k 10 200 python3 tools/kbench_fwd.py) > $O/kbench_$n.json 2>&1 || exit $?
  (cd $d && timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-epoch) > $O/bench_$n.log 2>&1 || exit $?
done
timeout -k 10 200 python3 tools/kbench_fwd.py > $O/kbench_head.json 2>&1 || exit $?
echo done
