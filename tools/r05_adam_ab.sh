set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for s in 1.0 0.25 0.02; do
  timeout -k 10 120 python3 tools/adam_micro.py $s 2>&1 | tail -1
  NGNN_ADAM_NO_TICKET=1 timeout -k 10 120 python3 tools/adam_micro.py $s 2>&1 | tail -1
done
