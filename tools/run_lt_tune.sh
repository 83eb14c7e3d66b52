# hipBLASLt candidate autotuning (NSTL_GEMM_LT_TUNE): the per-candidate times of
# the step's plain GEMM shapes, then the 228M step A/B tune on / off
set -o pipefail
cd $GRAFT_REPO_ROOT
NSTL_GEMM_LT_TUNE=2 timeout -k 10 300 python bench.py --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 --steps 5 --warmup 2 > gpurun_out/lt_tune.log 2>&1 || exit 1
grep "lt tune" gpurun_out/lt_tune.log | sort | uniq | head -80
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "hipblaslt" > gpurun_out/lt_tune_tests.log 2>&1 || exit 1
tail -1 gpurun_out/lt_tune_tests.log
bash tools/ab_env.sh NSTL_GEMM_LT_TUNE 3 1 0
