#!/bin/bash
# Build an A/B variant of libngnn.so with extra -D flags into ablib/<name>.so:
# the in-tree build's objects are reused, the row-tile kernel units are
# rebuilt with the flags.  usage: tools/build_variant.sh NAME "-DFOO=1 ..."
set -eu
cd "$(dirname "$0")/../noise-gnn_amd/csrc"
n=$1; shift
rm -rf build_$n && mkdir -p build_$n ../../ablib
cp -p build/*.o build_$n/
# (REBUILD: object stems to rebuild; default the row-tile kernel units)
for o in ${REBUILD:-ngnn_rt_* ngnn_sage_rt.hip ngnn_root.hip}; do rm -f build_$n/$o.o; done
make -s -j8 OBJ=build_$n OUT=../../ablib/_$n EXTRA="$*" >/dev/null
mv ../../ablib/_$n/libngnn.so ../../ablib/$n.so && rmdir ../../ablib/_$n
rm -rf build_$n
echo "built ablib/$n.so"
