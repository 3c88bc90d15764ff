#!/bin/bash
# eager loop host time by section with the C++ stack node (both Adams)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r06es}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 200 python3 tools/eager_sections.py --steps 300 > $O/torch_adam.txt 2>&1 || exit 3
timeout -k 10 200 python3 tools/eager_sections.py --steps 300 --ngnn-adam > $O/ngnn_adam.txt 2>&1 || exit 3
cat $O/torch_adam.txt $O/ngnn_adam.txt | grep -v amdgpu.ids
