#!/bin/bash
# Round 6, third batch: sampler / sync-free tests, the sampler alone under
# rocprofv3, the eager loop's cProfile, the headline bench (sync-free epoch)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06run3}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-loader or sample or sync_free}"
tail -3 $O/pytest.log
step sampler 200 rocprofv3 --kernel-trace --stats -d $O/prof_sampler -o run --output-format csv -- python3 tools/sampler_micro.py --blocks 40
python3 tools/sampler_micro.py --trace $O/prof_sampler/run_kernel_trace.csv > $O/sampler_trace.txt 2>&1
cat $O/sampler_trace.txt; grep wall $O/sampler.log
step eager_cprof 200 python3 tools/eager_step.py --cprofile
grep -v amdgpu $O/eager_cprof.log | head -50
step eager_sec 200 python3 tools/eager_sections.py
grep -v amdgpu $O/eager_sec.log
step bench_headline 400 python3 bench.py --no-cpu-baseline
tail -1 $O/bench_headline.log | cut -c1-300
step prof_epoch 400 rocprofv3 --kernel-trace --stats -d $O/prof_epoch -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eager-ref --timer none
python3 tools/epoch_trace.py $O/prof_epoch/run_kernel_trace.csv --batches 190 --skip-last 193 > $O/epoch_breakdown_sf.txt 2>&1
python3 tools/epoch_trace.py $O/prof_epoch/run_kernel_trace.csv --batches 190 --skip-last 386 > $O/epoch_breakdown_sync.txt 2>&1
python3 tools/epoch_trace.py $O/prof_epoch/run_kernel_trace.csv --batches 190 > $O/epoch_breakdown_fg.txt 2>&1
head -8 $O/epoch_breakdown_sf.txt $O/epoch_breakdown_sync.txt $O/epoch_breakdown_fg.txt
echo done
