#!/bin/bash
# One GPU call: the GPU test suite, smoke, the headline bench, its rocprof
# kernel stats, and the other configs' benches (BENCHES).  Each GPU step has
# its own time limit; a crash / abort / timeout ends the call there.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r03c}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {  # name timeout cmd...: stop the call on a crash / timeout (rc 1 = test failures: go on)
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  if [ -n "${PYTEST_K:-}" ]; then
    step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -k "$PYTEST_K"
  else
    step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread
  fi
  tail -3 $O/pytest_gpu.log
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 600 python3 bench.py ${BENCH_ARGS:---no-cpu-baseline}
tail -1 $O/bench.log | cut -c1-600
if [ "${SKIP_PROF:-0}" != 1 ]; then
  step prof 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --timer none
  python3 tools/trace_step.py $O/prof/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step_breakdown.txt 2>&1
  cat $O/step_breakdown.txt | head -20
fi
for b in ${BENCHES:-}; do
  case $b in
    gcn) step bench_gcn 300 python3 bench.py --no-cpu-baseline --module gcn ;;
    arxiv) step bench_arxiv 300 python3 bench.py --no-cpu-baseline --dataset ogbn-arxiv ;;
    computers) step bench_computers 300 python3 bench.py --no-cpu-baseline --dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max ;;
    p3_f32) step bench_p3_f32 400 python3 bench.py --no-cpu-baseline --fanout 20,15,10 --steps 20 --warmup 5 ;;
    p3_bf16) step bench_p3_bf16 400 python3 bench.py --no-cpu-baseline --fanout 20,15,10 --steps 20 --warmup 5 --dtype bf16 ;;
    fused) step bench_fused_gather 300 python3 bench.py --no-cpu-baseline --gather fused ;;
  esac
  tail -1 $O/bench_$b.log 2>/dev/null | cut -c1-300
done
echo done
