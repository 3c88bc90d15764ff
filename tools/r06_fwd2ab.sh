#!/bin/bash
# Round 6: k_fwd2 per-launch micro -- this tree vs ablib/libngnn_old.so (the
# round-5 kernel), then the attribution variants of the profiling build
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r06ab}; mkdir -p $O
timeout -k 10 200 python tools/fwd2_micro.py --stages main,fused --reps 50 > $O/micro_tree.log 2>&1 || exit 3
timeout -k 10 200 env NGNN_LIB=$PWD/ablib/libngnn_old.so python tools/fwd2_micro.py --stages main,fused --reps 50 > $O/micro_old.log 2>&1 || exit 4
timeout -k 10 300 env NGNN_LIB=$PWD/ablib/libngnn_dbg.so python tools/fwd2_micro.py --stages main --reps 50 --dbg ${DBGS:-1,2,3,4,8,16,5,12,15} > $O/micro_dbg.log 2>&1 || exit 5
tail -n 3 $O/micro_tree.log $O/micro_old.log; tail -n 12 $O/micro_dbg.log
