#!/bin/bash
# Round-end evidence: the whole GPU suite, smoke(), the default bench line
# (as the driver runs it), the headline's rocprof step breakdown, and the
# other configurations' bench lines
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06final}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  tail -1 $O/$n.log | cut -c1-250
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step pytest 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench_default 600 python3 bench.py
step prof_headline 400 rocprofv3 --kernel-trace --stats -d $O/prof_headline -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --no-eager-ref --timer none
python3 tools/trace_step.py $O/prof_headline/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step_headline.txt 2>&1
head -8 $O/step_headline.txt
for c in ${BENCHES:-computers gcn arxiv p3_ref coteaching}; do
  case $c in
    computers) A="--dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max" ;;
    arxiv) A="--dataset ogbn-arxiv" ;;
    arxiv5) A="--dataset ogbn-arxiv --fanout 10,5 --batch-size 512 --num-layers 3" ;;
    p3_bf16) A="--fanout 20,15,10 --dtype bf16 --steps 20 --warmup 5" ;;
    p3_ref) A="--fanout 15,10,5 --batch-size 512 --steps 20 --warmup 5" ;;
    gcn) A="--module gcn" ;;
    coteaching) A="--coteaching" ;;
  esac
  step bench_$c 400 python3 bench.py --no-cpu-baseline --no-eager-ref $A
done
echo done
