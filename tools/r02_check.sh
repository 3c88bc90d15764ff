#!/bin/bash
# Round-2 GPU check: tests, smoke, bench, rocprof kernel stats, PMC traffic of
# the two forward layer kernels on the bench workload (separate passes).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r02}
SKIP_PROF=1 TAG=$T bash tools/gpu_check.sh || exit $?
O=gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --timer none > "$O/prof.log" 2>&1
rc=$?; echo "[rocprof] rc=$rc" | tee -a $O/status.txt; [ $rc -ne 0 ] && exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex k_sage_rt -d "$O/pmc_$c" -o run --output-format csv -- python3 tools/kbench_fwd.py --reps 3 --only L0_model_x3,L1_model_x3 > "$O/pmc_$c.log" 2>&1
  rc=$?; echo "[pmc $c] rc=$rc" | tee -a $O/status.txt; [ $rc -ne 0 ] && exit $rc
done
echo done
