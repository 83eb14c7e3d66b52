# FFN dropout keep bits from the LayerNorm forward (NSTL_FFN_KEEP_LN): new tests,
# the kernel / model / production tests, then the FFN1 + LN kernel times and the
# 228M step A/B (switch on / off, one library)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_production_gpu.py tests/test_fp8_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "keep or relu or layernorm or gemm or production or bf16 or fp8" > gpurun_out/keep_tests.log 2>&1
rc=$?; tail -2 gpurun_out/keep_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh NSTL_FFN_KEEP_LN 3 1 0
