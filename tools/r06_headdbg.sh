#!/bin/bash
# the loss head's parts: narrow launch with the head, without its scatter
# (1), its loss hand-off (2), its cross entropy (4), and all three (7)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06hdbg}; O=gpurun_out/$T; mkdir -p $O
for pass in 1 2; do
  NGNN_LIB=$PWD/dbgh/libngnn_dbg.so timeout -k 10 200 python3 tools/fwd2_micro.py --stages narrow --head-dbg 1,2,4,7 --reps 50 > $O/micro_$pass.log 2>&1 || exit 3
  grep -E "^narrow" $O/micro_$pass.log | tee -a $O/summary.txt
done
