#!/bin/bash
# Round 6, fourth batch: the full GPU suite, the sampler alone, the headline
# bench (+ epoch breakdowns of its three epochs), config #4's DP line on gloo
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06run4}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
if [ "${FULL:-1}" = 1 ]; then
  NGNN_GRAD_LOG=$O/grad.jsonl step pytest 1500 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
  tail -3 $O/pytest.log
fi
step sampler 200 rocprofv3 --kernel-trace --stats -d $O/prof_sampler -o run --output-format csv -- python3 tools/sampler_micro.py --blocks 40
python3 tools/sampler_micro.py --trace $O/prof_sampler/run_kernel_trace.csv > $O/sampler_trace.txt 2>&1
cat $O/sampler_trace.txt
step bench_headline 400 python3 bench.py
tail -1 $O/bench_headline.log | cut -c1-300
step prof_epoch 400 rocprofv3 --kernel-trace --stats -d $O/prof_epoch -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eager-ref --timer none
python3 tools/epoch_trace.py $O/prof_epoch/run_kernel_trace.csv --batches 190 --skip-last 193 > $O/epoch_breakdown_sf.txt 2>&1
python3 tools/epoch_trace.py $O/prof_epoch/run_kernel_trace.csv --batches 190 --skip-last 386 > $O/epoch_breakdown_sync.txt 2>&1
python3 tools/epoch_trace.py $O/prof_epoch/run_kernel_trace.csv --batches 190 > $O/epoch_breakdown_fg.txt 2>&1
head -8 $O/epoch_breakdown_sf.txt $O/epoch_breakdown_sync.txt $O/epoch_breakdown_fg.txt
if [ "${DP:-1}" = 1 ]; then
  NGNN_DIST_BACKEND=gloo step bench_dp2_cfg4 600 python3 bench.py --gpus 2 --fanout 20,15,10 --dtype bf16 --steps 10 --warmup 3 --no-cpu-baseline --no-eager-ref --no-epoch
  tail -1 $O/bench_dp2_cfg4.log | cut -c1-300
fi
echo done
