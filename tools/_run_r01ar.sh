set -u
cd $GRAFT_REPO_ROOT
T=${TAG:-r01as}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_graphs_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$T/pytest.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/bench_kernels.py --reps 20 > gpurun_out/$T/kbench.json 2> gpurun_out/$T/kbench.err
echo "kbench rc=$?"
