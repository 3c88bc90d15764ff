#!/bin/bash
# Round-3 evidence, one GPU call: GPU tests + smoke, the headline bench (with
# the CPU baseline), its rocprof kernel stats / step breakdown, and PMC passes
# on the same bench command (FETCH_SIZE, WRITE_SIZE, the MFMA counters), one
# counter group per pass.  Each GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r03s}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_gpu 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  tail -2 $O/pytest_gpu.log
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  tail -1 $O/smoke.log
fi
step bench 600 python3 bench.py
tail -1 $O/bench.log | cut -c1-400
PB="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --timer none"
step prof 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- $PB
python3 tools/trace_step.py $O/prof/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step_breakdown.txt 2>&1
head -20 $O/step_breakdown.txt
PP="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-epoch --timer none"
i=0
IFS=';' read -ra GRPS <<< "${PMC_GROUPS:-FETCH_SIZE;WRITE_SIZE;SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAVES}"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  step pmc$i 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex 'k_sage_rt|k_root|k_x3_image' -d $O/pmc$i -o run --output-format csv -- $PP
done
python3 tools/pmc_summ.py $O k_ > $O/pmc_summary.txt 2>&1; cat $O/pmc_summary.txt | head -40
echo done
