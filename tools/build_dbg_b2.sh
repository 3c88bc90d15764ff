#!/bin/bash
# A profiling copy of libngnn.so with NGNN_B2_DBG_BUILD (k_bwd2's time-
# attribution variants, selected by NGNN_B2_DBG): dbgb/libngnn_dbg.so, used
# through NGNN_LIB by tools/bwd2_micro.py.  Never the product library.
set -e
cd "$(dirname "$0")/../noise-gnn_amd/csrc"
make -j8 >/dev/null
mkdir -p ../../dbgb
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -I../../include -I. \
  -DNGNN_B2_DBG_BUILD -c ngnn_bwd2.hip -o ../../dbgb/ngnn_bwd2_dbg.o
objs=$(ls build/*.o | grep -v ngnn_bwd2.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../dbgb/libngnn_dbg.so $objs ../../dbgb/ngnn_bwd2_dbg.o
rm ../../dbgb/ngnn_bwd2_dbg.o
echo built dbgb/libngnn_dbg.so
