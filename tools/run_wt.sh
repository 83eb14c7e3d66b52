# transposed bf16 weight copies for the input-gradient GEMMs (NSTL_WT): kernel,
# model and production-shape tests, then the 228M step A/B (alternating arms)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_production_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "transpose or production or bf16" > gpurun_out/wt_tests.log 2>&1
rc=$?; tail -3 gpurun_out/wt_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh NSTL_WT 3 1 0
