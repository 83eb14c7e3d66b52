set -o pipefail
cd $GRAFT_REPO_ROOT
for mode in fused persistent; do
  for nr in 0 1; do
    echo "--- $mode norope=$nr"; NSTL_BENCH_NOROPE=$nr NSTL_ATTN_BWD=$mode timeout -k 10 120 python tools/bench_attn.py || exit 1
  done
done
