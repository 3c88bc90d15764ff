#!/bin/bash
# Round-6 GPU call: optional pytest (ALL=1: every -m gpu test; PYTEST_K: a
# subset) with the gradient-error log, smoke, the benches in BENCHES (PROF=1:
# rocprof kernel stats + step breakdown each), DP=1: a two-rank gloo
# rehearsal of bench.py on the one GPU.  Each GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06x}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
if [ "${ALL:-0}" = 1 ]; then
  NGNN_GRAD_LOG=$O/grad.jsonl step pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  tail -3 $O/pytest.log
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  tail -1 $O/smoke.log
elif [ -n "${PYTEST_K:-}" ]; then
  NGNN_GRAD_LOG=$O/grad.jsonl step pytest 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "$PYTEST_K"
  tail -3 $O/pytest.log
fi
if [ "${DP:-0}" = 1 ]; then
  NGNN_DIST_BACKEND=gloo step dp2 400 python3 bench.py --gpus 2 --steps 20 --warmup 5 --scale 0.1 --no-cpu-baseline --no-epoch
  tail -1 $O/dp2.log | cut -c1-600
fi
for c in ${BENCHES:-}; do
  case $c in
    headline) A="" ;;
    fused) A="--gather fused" ;;
    eager) A="--eager" ;;
    computers) A="--dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max" ;;
    arxiv) A="--dataset ogbn-arxiv" ;;
    p3_f32) A="--fanout 20,15,10 --steps 20 --warmup 5" ;;
    p3_bf16) A="--fanout 20,15,10 --dtype bf16 --steps 20 --warmup 5" ;;
    p3_ref) A="--fanout 15,10,5 --batch-size 512 --steps 20 --warmup 5" ;;
    gcn) A="--module gcn" ;;
  esac
  step bench_$c 400 python3 bench.py --no-cpu-baseline $A
  tail -1 $O/bench_$c.log | cut -c1-300
  if [ "${PROF:-0}" = 1 ]; then
    step prof_$c 400 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --timer none $A
    python3 tools/trace_step.py $O/prof_$c/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step_$c.txt 2>&1
    head -24 $O/step_$c.txt
  fi
done
echo done
