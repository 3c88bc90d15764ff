#!/bin/bash
# Round 6, second batch: loader tests on the lane-per-draw sampler, the
# sampler alone under rocprofv3, the eager loop's host sections, config #3
# (bf16) and config_products-shape benches + config #3's HBM traffic passes.
# Every GPU step under its own time limit; stops at a crash.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06run2}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
if [ -n "${PYTEST_K:-}" ]; then
  step pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "$PYTEST_K"
  tail -3 $O/pytest.log
fi
if [ "${SAMPLER:-1}" = 1 ]; then
  step sampler 200 rocprofv3 --kernel-trace --stats -d $O/prof_sampler -o run --output-format csv -- python3 tools/sampler_micro.py --blocks 40
  python3 tools/sampler_micro.py --trace $O/prof_sampler/run_kernel_trace.csv > $O/sampler_trace.txt 2>&1
  cat $O/sampler_trace.txt; grep wall $O/sampler.log
fi
if [ "${EAGER:-1}" = 1 ]; then
  step eager_torch 200 python3 tools/eager_sections.py
  step eager_ngnn 200 python3 tools/eager_sections.py --ngnn-adam
  cat $O/eager_torch.log $O/eager_ngnn.log | grep -v amdgpu.ids
fi
for i in 1 2 3 4; do
  eval "A=\${BENCH_ARGS_$i:-}"
  if [ -n "$A" ]; then
    step bench_x$i 400 python3 bench.py --no-cpu-baseline $A
    tail -1 $O/bench_x$i.log | cut -c1-300
  fi
done
if [ -n "${PMC_ARGS:-}" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    step pmc_$c 300 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "${PMC_RE:-k_sage_rt}" -d $O/pmc_$c -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-epoch --no-eager-ref --timer none $PMC_ARGS
  done
fi
echo done
