#!/bin/bash
# the default bench line once more (the contract the driver runs)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r06bc}; mkdir -p $O
timeout -k 10 600 python3 bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 3; }
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['epoch_time_s'], d['eager_drop_in']['eager_cpp_node'], d['eager_drop_in']['ms_per_step'])"
