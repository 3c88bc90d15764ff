set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05mx}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "${K:-csr or wide or computers or max or configs or parity}" > $O/pytest.log 2>&1; echo "pytest rc=$? $(tail -1 $O/pytest.log)"
grep -E "^FAILED" $O/pytest.log | head -5
for v in 1 0; do
  NGNN_WIDE_X3=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-epoch --no-eager-ref --dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max > $O/bench_x3$v.log 2>&1 || exit 3
  echo "wide x3=$v $(tail -n1 $O/bench_x3$v.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
