# plain bf16 GEMMs on hipBLASLt (NSTL_GEMM_LT): GEMM + production tests, shape
# timings with it on/off, and the 228M step A/B (alternating arms)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_production_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "gemm or production or bf16 or fp32" > gpurun_out/lt_tests.log 2>&1
rc=$?; tail -3 gpurun_out/lt_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  echo "== NSTL_GEMM_LT=$v"; NSTL_GEMM_LT=$v timeout -k 10 200 python tools/bench_gemm_epi.py 2>/dev/null | grep -E "fwd out|fwd ffn2|dX  out|dX  ffn1 F32 beta1|dX  qkv|dX  q " || exit 1
done
bash tools/ab_env.sh NSTL_GEMM_LT 3 1 0
