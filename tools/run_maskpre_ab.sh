# dReLU mask words loaded before the K loop: GEMM/model tests, per-shape timings and the step, alternating NSTL_GEMM_MASKPRE
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_production_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/maskpre_tests.log 2>&1
rc=$?; tail -3 gpurun_out/maskpre_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for d in 0 1; do
    NSTL_GEMM_MASKPRE=$d timeout -k 10 200 python tools/bench_gemm_epi.py 2>/dev/null | grep -E "DRELU" | sed "s/^/P=$d: /" || exit 1
  done
done
bash tools/ab_env.sh NSTL_GEMM_MASKPRE 3 1 0
