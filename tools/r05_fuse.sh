#!/bin/bash
# k_fwd2x (edge + main phases in one launch): parity of the two-layer forward
# and the graph steps under it, then the headline bench alternating fused /
# two launches (NGNN_FWD2_FUSE=0), and a rocprof step breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05fz}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "fwd2 or head or configs or graph or gcn or fused or loader or dist or optim or fold" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-epoch > $O/bench_fz_$i.log 2>&1 || exit 1
  NGNN_FWD2_FUSE=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-epoch > $O/bench_two_$i.log 2>&1 || exit 1
  python3 -c "
import json
for n in ('fz','two'):
    d=json.loads(open('$O/bench_'+n+'_$i.log').read().strip().splitlines()[-1]); r=d['roofline']
    print(n, d['ms_per_step'], r['kernel'], r['avg_us'], r['frac'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --timer none > $O/prof.log 2>&1 || exit 1
python3 tools/trace_step.py $O/prof/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step_headline.txt 2>&1
head -9 $O/step_headline.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --no-epoch --dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max > $O/bench_computers.log 2>&1 || exit 1
tail -1 $O/bench_computers.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/profc -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --timer none --dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max > $O/profc.log 2>&1 || exit 1
python3 tools/trace_step.py $O/profc/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step_computers.txt 2>&1
head -20 $O/step_computers.txt
