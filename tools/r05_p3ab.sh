set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05wg2; mkdir -p $O
for v in 2 1; do
  NGNN_WGRAD_NFW=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-epoch --no-eager-ref --fanout 20,15,10 --dtype bf16 --steps 20 --warmup 5 > $O/bench_nfw$v.log 2>&1 || exit 3
  echo "nfw=$v $(tail -n1 $O/bench_nfw$v.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
NGNN_WGRAD_NFW=2 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-epoch --timer none --no-eager-ref --fanout 20,15,10 --dtype bf16 > $O/prof.log 2>&1 || exit 4
python3 tools/trace_step.py $O/prof/run_kernel_trace.csv --marker k_slot_load --skip 8 --steps 10 > $O/step.txt 2>&1
grep -E "span|wgrad" $O/step.txt
