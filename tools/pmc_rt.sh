#!/bin/bash
# PMC passes over the forward-kernel bench (tools/kbench_fwd.py): counter
# list, then one rocprofv3 --pmc pass per group (--kernel-trace only), each
# under its own time limit; stops at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-pmcrt}; mkdir -p $O
export TMPDIR=/tmp
CMD="python3 tools/kbench_fwd.py --reps 3 --only ${ONLY:-L0_noedges_x3,L0_model_x3}"
timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1
i=0
IFS=';' read -ra GRPS <<< "${GROUPS_PMC:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM}"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex k_sage_rt -d $O/pmc$i -o run --output-format csv -- $CMD > $O/pmc$i.log 2>&1
  rc=$?; echo "pmc$i ($grp) rc=$rc" | tee -a $O/status.txt
  [ $rc -ne 0 ] && { tail -3 $O/pmc$i.log; exit $rc; }
done
echo done
