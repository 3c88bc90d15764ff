#!/bin/bash
# bf16 row path: targeted tests, full GPU suite, config #3 both dtypes, headline.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-bf}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_graphs_gpu.py -k "bf16" -x -q --timeout 120 --timeout-method thread > $O/bf16_tests.log 2>&1 || { echo "bf16 tests rc=$?"; tail -30 $O/bf16_tests.log; exit 1; }
tail -1 $O/bf16_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python3 bench.py --no-cpu-baseline --fanout 20,15,10 --steps 20 --warmup 5 --dtype bf16 > $O/bench_p3_bf16.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --no-cpu-baseline --fanout 20,15,10 --steps 20 --warmup 5 > $O/bench_p3_f32.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
echo done
