#!/bin/bash
# k_wide_h2's XCD-aware tile order (default) vs the plain one
# (NGNN_WIDE_XCD=0): wide-path parity tests, the Computers bench alternating
# the two, and a step breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05wx}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "wide or computers or cora or 767 or k_not or pad" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
A="--dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max --no-cpu-baseline --no-epoch --no-eager-ref"
for i in 1 2; do
  timeout -k 10 300 python bench.py $A > $O/b_xcd_$i.log 2>&1 || exit 1
  NGNN_WIDE_XCD=0 timeout -k 10 300 python bench.py $A > $O/b_plain_$i.log 2>&1 || exit 1
  python3 -c "
import json
for n in ('xcd','plain'):
    d=json.loads(open('$O/b_'+n+'_$i.log').read().strip().splitlines()[-1]); print(n, d['ms_per_step'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --timer none $A > $O/prof.log 2>&1 || exit 1
python3 tools/trace_step.py $O/prof/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step.txt 2>&1
grep -E "k_wide|step span" $O/step.txt
