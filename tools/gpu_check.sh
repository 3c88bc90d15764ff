#!/bin/bash
# One gpurun call: GPU tests, smoke, a short bench and a rocprofv3 kernel-trace
# summary.  Every GPU step has its own time limit; a crash/abort/timeout stops
# the script (no further GPU work in the same call).  Test FAILURES (rc 1) do
# not stop it, so the bench still runs.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
stop_on_crash() {  # $1 = rc, $2 = step
  local rc=$1
  echo "[$2] rc=$rc" | tee -a "$OUT/status.txt"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $2 (rc=$rc)"; exit "$rc"; fi
}
rocm-smi --showproductname > "$OUT/gpu.txt" 2>&1 || true
nproc > "$OUT/host.txt"; lscpu | grep -E "Model name|^CPU\(s\)" >> "$OUT/host.txt" || true
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:--x} > "$OUT/pytest_gpu.log" 2>&1
  stop_on_crash $? pytest
  tail -5 "$OUT/pytest_gpu.log"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  stop_on_crash $? smoke
fi
if [ "${KBENCH:-0}" = 1 ]; then
  timeout -k 10 300 python3 tools/bench_kernels.py --reps 20 > "$OUT/kbench.json" 2> "$OUT/kbench.err"
  stop_on_crash $? kbench
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
  stop_on_crash $? bench
  tail -2 "$OUT/bench.log"
fi
if [ "${SKIP_PROF:-0}" != 1 ]; then
  timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py ${PROF_ARGS:---steps 20 --warmup 5 --no-cpu-baseline --no-epoch --timer none} > "$OUT/prof.log" 2>&1
  stop_on_crash $? rocprof
  find "$OUT/prof" -name "*kernel_stats.csv" -exec head -30 {} \; > "$OUT/kernel_stats_head.txt" 2>/dev/null || true
fi
echo done
