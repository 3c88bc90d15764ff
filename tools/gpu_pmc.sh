#!/bin/bash
# Kernel micro-benchmarks + PMC counter passes (one counter group per pass,
# --kernel-trace only: never combined with sys/runtime traces).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD=${PMC_CMD:-"python3 tools/bench_kernels.py --reps 5"}
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
timeout -k 10 300 python3 tools/bench_kernels.py --reps 20 > "$OUT/bench_kernels.json" 2> "$OUT/bench_kernels.err"
rc=$?; echo "bench_kernels rc=$rc"; [ $rc -ne 0 ] && exit $rc
i=0
PMC_GRP_LIST=${PMC_GROUPS:-"FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES;SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM;SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU"}
IFS=';' read -ra GRPS <<< "$PMC_GRP_LIST"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/pmc$i" -o run --output-format csv -- $CMD > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pmc$i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pmc$i.log"; fi
  if [ $rc -ge 124 ]; then exit $rc; fi
done
echo done
