set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05wd}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "wide or computers or max or configs" > $O/pytest.log 2>&1; echo "pytest rc=$? $(tail -1 $O/pytest.log)"
for v in 1 0; do
  NGNN_WIDE_X3=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-epoch --no-eager-ref --dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max > $O/bench_x3$v.log 2>&1 || exit 3
  echo "x3=$v $(tail -n1 $O/bench_x3$v.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --timer none --no-eager-ref --dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max > $O/prof.log 2>&1 || exit 4
python3 tools/trace_step.py $O/prof/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step.txt 2>&1
head -20 $O/step.txt | cut -c1-120
