#!/bin/bash
# k_bwd2 attribution: the micro on the product library and on the profiling
# build with constant chunk scales (NGNN_B2_DBG=1), kernel times by rocprof
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06b2}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  tail -2 $O/$n.log
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step micro_prod 120 python3 tools/bwd2_micro.py 100
NGNN_LIB=$PWD/dbgb/libngnn_dbg.so NGNN_B2_DBG=0 step micro_dbg0 120 python3 tools/bwd2_micro.py 100
NGNN_LIB=$PWD/dbgb/libngnn_dbg.so NGNN_B2_DBG=1 step micro_dbg1 120 python3 tools/bwd2_micro.py 100
export NGNN_LIB=$PWD/dbgb/libngnn_dbg.so
for d in 0 1; do
  export NGNN_B2_DBG=$d
  step prof_dbg$d 200 rocprofv3 --kernel-trace --stats -d $O/prof_dbg$d -o run --output-format csv -- python3 tools/bwd2_micro.py 50
  grep -h "k_bwd2<" $O/prof_dbg$d/run_kernel_stats.csv | cut -c1-200
done
echo done
