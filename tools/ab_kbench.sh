#!/bin/bash
# Forward-kernel A/B only: tools/kbench_fwd.py per library under ablib/
# (VARIANTS), the in-tree build first.  ONLY: kbench_fwd --only list.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-abk}; mkdir -p $O
for v in head ${VARIANTS:-}; do
  if [ $v = head ]; then unset NGNN_LIB; else export NGNN_LIB=$PWD/ablib/$v.so; fi
  timeout -k 10 200 python3 tools/kbench_fwd.py ${ONLY:+--only $ONLY} > $O/kbench_$v.json 2>&1 || exit $?
  echo "$v $(grep -v amdgpu.ids $O/kbench_$v.json | tr -d '\n ')"
done
echo done
