#!/bin/bash
# Round-4 evidence, one GPU call: GPU tests + smoke, the headline bench (with
# the CPU baseline), its rocprof kernel stats / step breakdown, PMC passes on
# the same bench command (FETCH_SIZE, WRITE_SIZE, MFMA counters; one counter
# group per pass), and the per-conv (INTEGRATION.md option A) kernel list.
# Each GPU step has its own time limit; SKIP_TESTS=1 / SKIP_PMC=1 skip parts.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r04f}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  tail -2 $O/pytest_gpu.log
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  tail -1 $O/smoke.log
fi
step bench 600 python3 bench.py ${BENCH_ARGS:-}
tail -1 $O/bench.log | cut -c1-600
PB="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --timer none"
step prof 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- $PB
python3 tools/trace_step.py $O/prof/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step_breakdown.txt 2>&1
head -24 $O/step_breakdown.txt
if [ "${SKIP_PMC:-0}" != 1 ]; then
  PP="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-epoch --timer none"
  i=0
  IFS=';' read -ra GRPS <<< "${PMC_GROUPS:-FETCH_SIZE;WRITE_SIZE;SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAVES;SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES}"
  for grp in "${GRPS[@]}"; do
    i=$((i+1))
    step pmc$i 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex 'k_fwd2|k_edge_nb|k_narrow_agg|k_wgrad|k_lowdim' -d $O/pmc$i -o run --output-format csv -- $PP
  done
  python3 tools/pmc_summ.py $O k_ > $O/pmc_summary.txt 2>&1; head -60 $O/pmc_summary.txt
fi
if [ "${PERCONV:-1}" = 1 ]; then
  step perconv 300 rocprofv3 --kernel-trace --stats -d $O/perconv -o run --output-format csv -- python3 tools/perconv_step.py
  python3 tools/kstats.py $O/perconv/run_kernel_stats.csv > $O/perconv_kernels.txt 2>&1 || cp $O/perconv/run_kernel_stats.csv $O/perconv_kernels.txt
  n=$(grep -ciE "cijk|rocblas|hipblaslt|tensile" $O/perconv/run_kernel_stats.csv || true)
  echo "library GEMM kernels (Cijk / rocBLAS / hipBLASLt / Tensile) in the step: $n" >> $O/perconv_kernels.txt
  head -40 $O/perconv_kernels.txt
fi
echo done
