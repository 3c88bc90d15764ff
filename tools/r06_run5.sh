#!/bin/bash
# Round 6, config benches: the full GPU suite, then each named bench line and
# its rocprof step breakdown (tools/trace_step.py)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06run5}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
if [ "${FULL:-1}" = 1 ]; then
  step pytest 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
  tail -1 $O/pytest.log
fi
for c in ${BENCHES:-computers}; do
  case $c in
    headline) A="" ;;
    computers) A="--dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max" ;;
    arxiv) A="--dataset ogbn-arxiv" ;;
    arxiv5) A="--dataset ogbn-arxiv --fanout 10,5 --batch-size 512 --num-layers 3" ;;
    p3_bf16) A="--fanout 20,15,10 --dtype bf16 --steps 20 --warmup 5" ;;
    p3_ref) A="--fanout 15,10,5 --batch-size 512 --steps 20 --warmup 5" ;;
    gcn) A="--module gcn" ;;
    coteaching) A="--coteaching" ;;
  esac
  step bench_$c 400 python3 bench.py --no-cpu-baseline $A
  tail -1 $O/bench_$c.log | cut -c1-250
  if [ "${PROF:-1}" = 1 ]; then
    step prof_$c 400 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --no-eager-ref --timer none $A
    python3 tools/trace_step.py $O/prof_$c/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step_$c.txt 2>&1
    head -3 $O/step_$c.txt
  fi
done
echo done
