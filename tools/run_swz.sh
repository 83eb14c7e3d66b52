# LDS swizzle check: GEMM/model parity, LDS counters, bench A/B vs libnstl_hip_old.so
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_model_gpu.py > gpurun_out/swz_tests.log 2>&1 || { tail -30 gpurun_out/swz_tests.log; exit 1; }
tail -3 gpurun_out/swz_tests.log
bash tools/run_pmc_lds.sh || exit 1
cd $R && bash tools/ab_lib.sh 2
