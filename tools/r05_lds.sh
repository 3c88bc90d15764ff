#!/bin/bash
# k_fwd2 LDS experiment: parity of the two-layer forward, the main launch's
# LDS bank conflicts (PMC) and its time in the fwd2 micro, a headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05lds}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "fwd2 or headline or gcn or head" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
g="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $g --kernel-include-regex "k_fwd2<" -d $O/s -o run --output-format csv -- python3 tools/fwd2_micro.py --stages main --reps 10 > $O/s.log 2>&1 || { tail -3 $O/s.log; exit 1; }
for i in 1 2; do timeout -k 10 120 python3 tools/fwd2_micro.py --stages main,fused --reps 50 > $O/micro$i.log 2>&1 || exit 1; tail -2 $O/micro$i.log; done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-epoch --no-eager-ref > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | cut -c1-200
