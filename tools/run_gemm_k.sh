# K-scaling of the ring GEMM at N = 1024 (one round) and 4096 (four rounds), with
# the epilogue on, with the global stores skipped, and with the whole epilogue skipped
set -o pipefail
cd $GRAFT_REPO_ROOT
for n in 1024 4096; do
  for mode in none skip_store skip_epi; do
    echo "== N=$n epilogue mode $mode"
    NSTL_GEMM_DEBUG=$mode timeout -k 10 200 python tools/bench_gemm_k.py $n 0 2>/dev/null | grep -v amdgpu || exit 1
  done
done
