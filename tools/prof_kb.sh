#!/bin/bash
# rocprof kernel stats of kbench_fwd cases per library (head + VARIANTS under ablib/)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-pkb}; mkdir -p $O
export TMPDIR=/tmp
for v in head ${VARIANTS:-}; do
  if [ $v = head ]; then unset NGNN_LIB; else export NGNN_LIB=$PWD/ablib/$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 tools/kbench_fwd.py --reps 5 ${ONLY:+--only $ONLY} > $O/$v.log 2>&1 || exit $?
  echo "== $v"; python3 - "$O/$v" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:60]:60s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:8.2f}")
PY
done
