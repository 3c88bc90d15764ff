#!/bin/bash
# Round-5 final benches: the eager loop's host profile (cProfile, ngnn Adam),
# then the configs with rocprof step breakdowns (tools/r05_run.sh).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05bn}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/eager_step.py --steps 30 --ngnn-adam --cprofile > $O/eager_prof.log 2>&1 || exit 1
head -3 $O/eager_prof.log
