#!/bin/bash
# PMC passes over tools/fwd2_micro.py (k_fwd2 / k_edge_nb; optional DBG
# variants through the profiling library).  One counter group per pass.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r04pm}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
GROUPS_DEF="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM"
MICRO=${MICRO:-"tools/fwd2_micro.py --reps 10 --stages ${STAGES:-main} --dbg=${DBGS:-}"}
IFS=';' read -ra GRPS <<< "${PMC_GROUPS:-$GROUPS_DEF}"
i=0
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "${KRE:-k_fwd2|k_edge_nb}" -d $O/pmc$i -o run --output-format csv -- python3 $MICRO > $O/pmc$i.log 2>&1
  rc=$?; echo "[pmc$i] rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 tools/pmc_summ.py $O k_ > $O/pmc_summary.txt 2>&1; cat $O/pmc_summary.txt
