#!/bin/bash
# 1-GPU headline bench under several env settings on one box (A/B of host
# policies): CASES="name:VAR=val,VAR=val name2:..." ; "base" = no overrides
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-abe}; mkdir -p $O
for rep in 1 2; do
for c in ${CASES}; do
  n=${c%%:*}; kv=${c#*:}
  envs=""; [ "$kv" != "$n" ] && envs=$(echo "$kv" | tr ',' ' ')
  env $envs timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-epoch ${ARGS:-} > $O/bench_${n}_$rep.log 2>&1 || exit $?
  echo "$n rep$rep $(tail -1 $O/bench_${n}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_us"])')"
done
done
