#!/bin/bash
# run one GPU test selection R times with each library of LIBS (in-tree build: "tree")
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05fl}; mkdir -p $O
for v in $LIBS; do
  if [ $v = tree ]; then L=""; else L=$PWD/ablib/libngnn_$v.so; fi
  for r in $(seq ${R:-3}); do
    NGNN_LIB=$L timeout -k 10 300 python -u -m pytest ${F:-tests/test_gpu_fwd2.py} -m gpu -q --timeout 200 --timeout-method thread -k "${K:-many_tiles}" > $O/${v}_$r.log 2>&1
    rc=$?; echo "$v run$r rc=$rc $(tail -1 $O/${v}_$r.log)" | tee -a $O/summary.txt
    if [ $rc -gt 1 ]; then exit $rc; fi
  done
done
