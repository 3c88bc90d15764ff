#!/bin/bash
# LDS bank conflicts of k_fwd2 under its time-attribution variants
# (NGNN_FWD2_DBG bits on the profiling build, tools/build_dbg.sh): which part
# of a step holds the conflicts.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05pmc5}; mkdir -p $O
export TMPDIR=/tmp
g="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS"
for v in 0 1 2 4 8 16; do
  NGNN_LIB=dbg/libngnn_dbg.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $g --kernel-include-regex "k_fwd2<" -d $O/v$v -o run --output-format csv -- python3 tools/fwd2_micro.py --stages main --dbg $v --reps 5 > $O/v$v.log 2>&1 || { tail -3 $O/v$v.log; exit 1; }
done
echo done
