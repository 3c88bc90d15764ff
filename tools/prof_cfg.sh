#!/bin/bash
# rocprof kernel trace + per-step breakdown of the non-headline configs (CFGS)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r03g}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for c in ${CFGS:-computers p3_bf16}; do
  case $c in
    computers) A="--dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max" ;;
    arxiv) A="--dataset ogbn-arxiv" ;;
    p3_f32) A="--fanout 20,15,10" ;;
    p3_bf16) A="--fanout 20,15,10 --dtype bf16" ;;
    gcn) A="--module gcn" ;;
  esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --timer none $A > $O/prof_$c.log 2>&1
  rc=$?; echo "[$c] rc=$rc" | tee -a $O/status.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
  python3 tools/trace_step.py $O/prof_$c/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step_$c.txt 2>&1
  head -30 $O/step_$c.txt
done
