set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r01bh; mkdir -p $O
timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "rowtile or sage or fused" > $O/pytest.log 2>&1; echo "pytest rc=$?" >> $O/status.txt
NGNN_RT_MAXNTW=8 timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "rowtile or sage or fused" > $O/pytest_ntw8.log 2>&1; rc=$?; echo "pytest8 rc=$rc" >> $O/status.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-epoch > $O/bench16.log 2>&1 || exit $?
NGNN_RT_MAXNTW=8 timeout -k 10 300 python bench.py --no-cpu-baseline --no-epoch > $O/bench8.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --no-epoch > $O/bench16b.log 2>&1 || exit $?
tail -1 $O/pytest.log $O/pytest_ntw8.log
for f in bench16 bench8 bench16b; do grep -o '"ms_per_step": [0-9.]*' $O/$f.log; grep -o '"sage_fwd_l0": {[^}]*}' $O/$f.log; done
