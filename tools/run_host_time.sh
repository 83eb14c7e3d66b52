# host enqueue cost of the step with hipBLASLt on and off
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 1 0; do
  echo "== NSTL_GEMM_LT=$v"; NSTL_GEMM_LT=$v timeout -k 10 300 python tools/host_time.py 2>/dev/null || exit 1
done
