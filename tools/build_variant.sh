#!/bin/bash
# Build an A/B variant of libngnn.so with extra -D flags into ablib/<name>.so
# usage: tools/build_variant.sh NAME "-DFOO=1 ..."
set -eu
cd "$(dirname "$0")/../noise-gnn_amd/csrc"
n=$1; shift
mkdir -p ../../ablib build_$n
for f in *.hip *.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -I../../include -I. "$@" -c $f -o build_$n/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../ablib/$n.so build_$n/*.o
rm -rf build_$n
