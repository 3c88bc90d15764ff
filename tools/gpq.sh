#!/bin/bash
# queue a gpurun call: retries ONLY while gpurun reports no free box / slot
# (exit 3 or status=transient: nothing ran, nothing charged), every 150 s
OUT=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun "$@" > $OUT 2>&1; rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" $OUT; then sleep 150; continue; fi
  echo "rc=$rc" >> $OUT; echo done >> $OUT; exit 0
done
echo "gave up" >> $OUT
