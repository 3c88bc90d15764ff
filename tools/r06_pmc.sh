#!/bin/bash
# SQ counters of the fused two-layer forward (k_fwd2x) and k_bwd2 on the
# headline block: one counter group per rocprofv3 pass (--kernel-trace only).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r06pmc}; mkdir -p $O
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM" "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "k_fwd2x" -d $O/f$i -o run --output-format csv -- python3 tools/fwd2_micro.py --stages fused --reps 10 > $O/f$i.log 2>&1 || { echo "f$i failed"; tail -3 $O/f$i.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "k_bwd2<" -d $O/b$i -o run --output-format csv -- python3 tools/bwd2_micro.py 10 > $O/b$i.log 2>&1 || { echo "b$i failed"; tail -3 $O/b$i.log; exit 1; }
done
echo sq done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "k_fwd2x|k_narrow_agg" -d $O/pmc_$c -o run --output-format csv -- python3 tools/fwd2_micro.py --stages fused,narrow --head --reps 10 > $O/pmc_$c.log 2>&1 || { tail -5 $O/pmc_$c.log; exit 1; }
done
echo traffic done
