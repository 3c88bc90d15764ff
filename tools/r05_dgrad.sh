#!/bin/bash
# k_dgrad_fused for a narrow W (F_out < 32) from L2 (default) vs staged in
# LDS (NGNN_DGRAD_LDSW=1): the dgrad / computers / cora parity tests under
# the default, the Computers bench alternating the two, a step breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05dg}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "dgrad or backward or bwd or computers or cora or max or wide" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
A="--dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max --no-cpu-baseline --no-epoch --no-eager-ref"
for i in 1 2; do
  timeout -k 10 300 python bench.py $A > $O/b_l2_$i.log 2>&1 || exit 1
  NGNN_DGRAD_LDSW=1 timeout -k 10 300 python bench.py $A > $O/b_lds_$i.log 2>&1 || exit 1
  python3 -c "
import json
for n in ('l2','lds'):
    d=json.loads(open('$O/b_'+n+'_$i.log').read().strip().splitlines()[-1]); print(n, d['ms_per_step'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --timer none $A > $O/prof.log 2>&1 || exit 1
python3 tools/trace_step.py $O/prof/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step.txt 2>&1
grep -E "k_dgrad|k_dh_init|step span" $O/step.txt
