#!/bin/bash
# k_adam on Amazon-Computers' parameters: graph-timed micro and rocprof
# kernel durations for the ticket / no-ticket forms and per-CU caps
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06am}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "[$n] rc=$rc" | tee -a $O/status.txt
  grep -h "us/launch" $O/$n.log | tail -1
  if [ $rc -ne 0 ]; then exit $rc; fi
}
for cfg in "def:" "nt:NGNN_ADAM_NO_TICKET=1" "w1:NGNN_ADAM_WG_PER_CU=1" "w4:NGNN_ADAM_WG_PER_CU=4" "w8:NGNN_ADAM_WG_PER_CU=8"; do
  n=${cfg%%:*}; e=${cfg#*:}
  if [ -n "$e" ]; then export "$e"; fi
  step micro_$n 120 python3 tools/adam_micro.py
  step prof_$n 120 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run --output-format csv -- python3 tools/adam_micro.py
  python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_$n/run_kernel_stats.csv')):
    if 'adam' in r['Name'] or 'step_inc' in r['Name']: print('   ', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')"
  if [ -n "$e" ]; then unset "${e%%=*}"; fi
done
echo done
