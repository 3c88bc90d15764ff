#!/bin/bash
# Computers / config #3 after the weight gradient's XCD-grouped grid and the
# Adam launch change: their parity tests, benches and step breakdowns.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05cmp}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "wgrad or optim or fold or computers or p3 or 3layer or cora or perconv or stack" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
TAG=${TAG:-r05cmp} BENCHES="computers p3_bf16" PROF=1 bash tools/r05_run.sh
