#!/bin/bash
# build_variant.sh NAME "DEFINES" [SRC]: libngnn with SRC (default ngnn_fwd2.hip)
# recompiled under DEFINES, into ablib/libngnn_NAME.so (A/B experiments)
set -e
cd "$(dirname "$0")/../noise-gnn_amd/csrc"
N=$1; D=$2; S=${3:-ngnn_fwd2.hip}
mkdir -p /tmp/abobj_$N
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -I../../include -I. $D -c $S -o /tmp/abobj_$N/$S.o
OBJS=$(ls build/*.o | grep -v "build/$S.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../ablib/libngnn_$N.so $OBJS /tmp/abobj_$N/$S.o
echo built ablib/libngnn_$N.so
