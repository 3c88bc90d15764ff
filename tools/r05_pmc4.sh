set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05pmc4; mkdir -p $O
export TMPDIR=/tmp
g="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $g --kernel-include-regex "k_edge_nb|k_fwd2<" -d $O/s -o run --output-format csv -- python3 tools/fwd2_micro.py --stages edge,main --reps 10 > $O/s.log 2>&1 || { tail -3 $O/s.log; exit 1; }
echo done
