#!/bin/bash
# Round-end evidence in one call: GPU tests, smoke, the headline bench (with
# CPU baseline), its rocprof kernel stats, PMC traffic of the L0 forward,
# the other BASELINE configs and the forward kernel bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r02z}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {  # name timeout cmd...: stop the call on a crash / timeout
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
tail -1 $O/pytest_gpu.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
step prof 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --timer none
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c 180 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex k_sage_rt -d $O/pmc_$c -o run --output-format csv -- python3 tools/kbench_fwd.py --reps 3 --only L0_model_x3,L1_model_x3
done
step bench_gcn 300 python3 bench.py --no-cpu-baseline --module gcn
step bench_fused_gather 300 python3 bench.py --no-cpu-baseline --gather fused
step bench_arxiv 300 python3 bench.py --no-cpu-baseline --dataset ogbn-arxiv
step bench_computers 300 python3 bench.py --no-cpu-baseline --dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max
step bench_p3_f32 400 python3 bench.py --no-cpu-baseline --fanout 20,15,10 --steps 20 --warmup 5
step bench_p3_bf16 400 python3 bench.py --no-cpu-baseline --fanout 20,15,10 --steps 20 --warmup 5 --dtype bf16
step kbench 300 python3 tools/kbench_fwd.py
echo done
