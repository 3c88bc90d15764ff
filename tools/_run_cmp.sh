set -u
cd $GRAFT_REPO_ROOT
T=${TAG:-cmp}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_graphs_gpu.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$T/pytest.log
if [ $rc -gt 1 ]; then exit $rc; fi
for v in ${VARIANTS:-X=0 NGNN_SPLIT=2 NGNN_SPLIT=1 X=1}; do
  env $v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-epoch > gpurun_out/$T/bench_$v.log 2>&1
  echo "bench $v rc=$?"; tail -1 gpurun_out/$T/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], {k: v['avg_us'] for k, v in d['roofline']['all_kernels'].items()})"
done
if [ "${PROF:-0}" = 1 ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --timer none > gpurun_out/$T/prof.log 2>&1
  echo "prof rc=$?"
fi
