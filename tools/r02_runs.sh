#!/bin/bash
# GPU tests + forward kernel bench + the bench lines of the BASELINE configs.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r02}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 tools/kbench_fwd.py > $O/kbench.json 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline --module gcn > $O/bench_gcn.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline --gather loader > $O/bench_loadergather.log 2>&1 || exit $?
if [ "${CONFIGS:-0}" = 1 ]; then
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --dataset ogbn-arxiv > $O/bench_arxiv.log 2>&1 || exit $?
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max > $O/bench_computers.log 2>&1 || exit $?
  timeout -k 10 400 python3 bench.py --no-cpu-baseline --fanout 20,15,10 --steps 20 --warmup 5 > $O/bench_p3_f32.log 2>&1 || exit $?
  timeout -k 10 400 python3 bench.py --no-cpu-baseline --fanout 20,15,10 --steps 20 --warmup 5 --dtype bf16 > $O/bench_p3_bf16.log 2>&1 || exit $?
fi
echo done
