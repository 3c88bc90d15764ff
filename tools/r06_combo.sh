#!/bin/bash
# Round 6 combined GPU call: tests (PYTEST_K), headline bench + its rocprof
# step breakdown, the epoch trace, micro A/B over LIBS, extra bench lines
# (BENCH_ARGS_n), each step under its own time limit; stops at a crash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06x}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
if [ -n "${PYTEST_K:-}" ]; then
  NGNN_GRAD_LOG=$O/grad.jsonl step pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "$PYTEST_K"
  tail -3 $O/pytest.log
fi
if [ "${HEADLINE:-1}" = 1 ]; then
  step bench_headline 400 python3 bench.py --no-cpu-baseline
  tail -1 $O/bench_headline.log | cut -c1-400
  step prof_headline 400 rocprofv3 --kernel-trace --stats -d $O/prof_headline -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --timer none
  python3 tools/trace_step.py $O/prof_headline/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step_headline.txt 2>&1
  head -12 $O/step_headline.txt
  step prof_epoch 400 rocprofv3 --kernel-trace --stats -d $O/prof_epoch -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eager-ref --timer none
  python3 tools/epoch_trace.py $O/prof_epoch/run_kernel_trace.csv --batches 190 > $O/epoch_breakdown.txt 2>&1
  head -30 $O/epoch_breakdown.txt
fi
if [ -n "${LIBS:-}" ]; then
  for v in $LIBS; do
    if [ $v = tree ]; then L=""; else L=$PWD/ablib/libngnn_$v.so; fi
    NGNN_LIB=$L step micro_$v 200 python tools/fwd2_micro.py --stages main,fused --reps 50
    echo "$v $(grep -E '^(main|fused) ' $O/micro_$v.log | tr -s ' ' | cut -d' ' -f1,2 | tr '\n' ' ')" | tee -a $O/summary.txt
  done
fi
for i in 1 2 3 4; do
  eval "A=\${BENCH_ARGS_$i:-}"
  if [ -n "$A" ]; then
    step bench_x$i 400 python3 bench.py --no-cpu-baseline $A
    tail -1 $O/bench_x$i.log | cut -c1-500
  fi
done
echo done
