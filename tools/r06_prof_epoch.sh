#!/bin/bash
# Round 6: rocprof kernel trace of a short bench.py run whose last phase is
# the epoch (193 batches incl. GPU sampling); tools/epoch_trace.py splits it
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06e}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_epoch -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eager-ref --timer none ${EXTRA:-} > $O/prof_epoch.log 2>&1 || exit $?
tail -1 $O/prof_epoch.log | cut -c1-400
python3 tools/epoch_trace.py $O/prof_epoch/run_kernel_trace.csv --batches 190 > $O/epoch_breakdown.txt 2>&1
cat $O/epoch_breakdown.txt | head -40
