#!/bin/bash
# PMC counter passes over tools/kbench_fwd.py (one counter group per pass,
# --kernel-trace only), limited to the row-tile forward kernel.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-pmcfwd}
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD="python3 tools/kbench_fwd.py --reps 3 --only ${ONLY:-L0_model_x3}"
timeout -k 10 300 python3 tools/kbench_fwd.py > "$OUT/kbench.json" 2> "$OUT/kbench.err"
rc=$?; echo "kbench rc=$rc"; [ $rc -ne 0 ] && exit $rc
i=0
PMC_GRP_LIST=${PMC_GROUPS:-"SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES;SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM;SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU;FETCH_SIZE;WRITE_SIZE"}
IFS=';' read -ra GRPS <<< "$PMC_GRP_LIST"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "k_sage_rt" -d "$OUT/pmc$i" -o run --output-format csv -- $CMD > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pmc$i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pmc$i.log"; exit $rc; fi
done
echo done
