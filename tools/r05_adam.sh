#!/bin/bash
# Adam's first-chunk prefetch: the optimiser tests, tools/adam_micro.py and
# the Computers bench (its layer-by-layer step runs k_adam), with a step
# breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05adam}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "adam or optim" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python tools/adam_micro.py > $O/micro.log 2>&1 || { tail -20 $O/micro.log; exit 1; }
tail -5 $O/micro.log
A="--dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max --no-cpu-baseline --no-epoch --no-eager-ref"
for i in 1 2; do
  timeout -k 10 300 python bench.py $A > $O/b_$i.log 2>&1 || exit 1
  python3 -c "import json; print(json.loads(open('$O/b_$i.log').read().strip().splitlines()[-1])['ms_per_step'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --timer none $A > $O/prof.log 2>&1 || exit 1
python3 tools/trace_step.py $O/prof/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step.txt 2>&1
grep -E "k_adam|step span" $O/step.txt
