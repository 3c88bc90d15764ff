#!/bin/bash
# A/B of k_fwd2 builds: fwd2 parity tests on the in-tree build, then the
# per-launch micro on each library in LIBS (default: ablib/libngnn_base.so
# and the in-tree build), then optionally the headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r05ab}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
if [ -n "${PYTEST_K:-}" ]; then
  step pytest 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread ${PYTEST_F:-tests/test_gpu_fwd2.py} -k "$PYTEST_K"
  tail -3 $O/pytest.log
fi
i=0
for L in ${LIBS:-ablib/libngnn_base.so noise-gnn_amd/ngnn/lib/libngnn.so}; do
  NGNN_LIB=$PWD/$L step micro$i 300 python tools/fwd2_micro.py --stages ${STAGES:-main} --reps 50
  grep -E "main|edge|narrow" $O/micro$i.log | tail -3
  i=$((i+1))
done
if [ "${BENCH:-0}" = 1 ]; then
  step bench 300 python bench.py --no-cpu-baseline --no-epoch --no-eager-ref
  tail -1 $O/bench.log | cut -c1-400
fi
