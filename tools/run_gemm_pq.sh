# The persistent cross-tile pipelined GEMM (NSTL_GEMM_PQ=1; 2 also runs single-
# round problems on it, a diagnostic of its K loop): GEMM tests with it on, then
# the epilogue-shape timings alternating off / on.
set -o pipefail
cd $GRAFT_REPO_ROOT
NSTL_GEMM_PQ=1 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/pq_tests.log 2>&1
rc=$?; tail -3 gpurun_out/pq_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in 0 1; do
  echo "== NSTL_GEMM_PQ=$v"; NSTL_GEMM_PQ=$v timeout -k 10 200 python tools/bench_gemm_epi.py 2>/dev/null | grep -E "fwd ffn1 BIAS|dX  ffn2 bf16|fwd out|fwd ffn2|dX  out" || exit 1
done; done
