#!/bin/bash
# k_bwd2 A/B: the weight slice's loads overlapping the first chunk's (tree)
# against abv/libngnn_b2old.so (split first); micro + rocprof + bwd2 tests
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06b2p}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bwd2.py tests/test_gpu_fold.py -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
for pass in 1 2; do
  for v in tree b2old; do
    if [ $v = tree ]; then L=""; else L=$PWD/abv/libngnn_$v.so; fi
    NGNN_LIB=$L timeout -k 10 200 python3 tools/bwd2_micro.py 100 > $O/b2_${v}_$pass.log 2>&1 || exit 3
    echo "$pass $v $(grep us/call $O/b2_${v}_$pass.log)" | tee -a $O/summary.txt
  done
done
for v in tree b2old; do
  if [ $v = tree ]; then L=""; else L=$PWD/abv/libngnn_$v.so; fi
  NGNN_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 tools/bwd2_micro.py 50 > $O/prof_$v.log 2>&1 || exit 3
  python3 -c "
import csv
for r in csv.DictReader(open('$O/prof_$v/run_kernel_stats.csv')):
    if 'k_bwd2<' in r['Name']: print('$v', r['Name'][:40], round(float(r['AverageNs'])/1e3,2), 'us')" | tee -a $O/summary.txt
done
echo done
