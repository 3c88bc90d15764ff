#!/bin/bash
# A profiling copy of libngnn.so with NGNN_FWD2_DBG_BUILD (k_fwd2's time-
# attribution variants, selected by NGNN_FWD2_DBG): dbg/libngnn_dbg.so, used
# through NGNN_LIB by tools/fwd2_micro.py.  Never the product library.
set -e
cd "$(dirname "$0")/../noise-gnn_amd/csrc"
make -j8 >/dev/null
mkdir -p ../../dbg
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -I../../include -I. \
  -DNGNN_FWD2_DBG_BUILD -c ngnn_fwd2.hip -o ../../dbg/ngnn_fwd2_dbg.o
objs=$(ls build/*.o | grep -v ngnn_fwd2.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../dbg/libngnn_dbg.so $objs ../../dbg/ngnn_fwd2_dbg.o
rm ../../dbg/ngnn_fwd2_dbg.o
echo built dbg/libngnn_dbg.so
