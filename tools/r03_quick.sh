#!/bin/bash
# Quick GPU check: GPU tests, then the computers config and the headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-q}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {  # name timeout cmd...: stop the call on a crash / timeout
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
tail -1 $O/pytest_gpu.log
for b in ${BENCHES:-computers headline}; do
  case $b in
    computers) step bench_computers 300 python3 bench.py --no-cpu-baseline --dataset computers --fanout 10,5 --batch-size 300 --hidden 512 --aggr max ;;
    headline) step bench_headline 300 python3 bench.py --no-cpu-baseline ;;
    p3_f32) step bench_p3_f32 400 python3 bench.py --no-cpu-baseline --fanout 20,15,10 --steps 20 --warmup 5 ;;
    p3_bf16) step bench_p3_bf16 400 python3 bench.py --no-cpu-baseline --fanout 20,15,10 --steps 20 --warmup 5 --dtype bf16 ;;
  esac
  tail -1 $O/bench_$b.log 2>/dev/null | cut -c1-400
done
echo done
