#!/bin/bash
# rocprof kernel stats of the 3-layer products configs (fp32 and bf16 models).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-p3prof}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for dt in ${DTYPES:-f32 bf16}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$dt -o run --output-format csv -- python3 bench.py --fanout 20,15,10 --steps 10 --warmup 3 --no-cpu-baseline --no-epoch --timer none --dtype $dt > $O/prof_$dt.log 2>&1
  rc=$?; echo "[prof_$dt] rc=$rc" | tee -a $O/status.txt; [ $rc -ne 0 ] && exit $rc
done
echo done
