#!/bin/bash
# The other BASELINE.json configs through bench.py (the headline line is
# configs[1]'s metric on products-[15,10]; these are the supplementary
# measurements DESIGN.md reports).  One process per config, each bounded.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-configs}; mkdir -p "$OUT"
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-400
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  return 0
}
run arxiv_15_10_f32 --dataset ogbn-arxiv
run products_20_15_10_bf16 --fanout 20,15,10 --dtype bf16
run products_20_15_10_f32 --fanout 20,15,10
run computers_10_5_max --dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max
echo done
