#!/bin/bash
# dump ngnn_sage2_fwd outputs with ablib/libngnn_base.so and each variant in
# VARS (ablib/libngnn_<v>.so; "tree": the in-tree build), compare to base
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r05ab3}; mkdir -p $O
NGNN_LIB=$PWD/ablib/libngnn_base.so timeout -k 10 200 python tools/ab_fwd2_dump.py /tmp/base.pt > $O/dump_base.log 2>&1 || exit 3
for v in $VARS; do
  if [ $v = tree ]; then L=""; else L=$PWD/ablib/libngnn_$v.so; fi
  NGNN_LIB=$L timeout -k 10 200 python tools/ab_fwd2_dump.py /tmp/$v.pt > $O/dump_$v.log 2>&1 || exit 4
  echo "== $v" >> $O/cmp.txt
  python tools/ab_fwd2_cmp.py /tmp/base.pt /tmp/$v.pt >> $O/cmp.txt
done
cat $O/cmp.txt
