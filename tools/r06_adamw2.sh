#!/bin/bash
# k_adam per-CU workgroup cap with the ABI-21 line-spread ticket: graph micro
# (Computers' parameters) and rocprof kernel time per cap
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06aw2}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for pass in 1 2; do
  for w in 1 2 4; do
    NGNN_ADAM_WG_PER_CU=$w timeout -k 10 120 python3 tools/adam_micro.py > $O/m_${w}_$pass.log 2>&1 || exit 3
    echo "$pass w=$w $(grep us/launch $O/m_${w}_$pass.log)" | tee -a $O/summary.txt
  done
done
echo done
