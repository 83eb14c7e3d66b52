set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gemm4_gpu.py tests/test_tight_parity_gpu.py tests/test_kernels_gpu.py tests/test_fp8_gpu.py -q -x --timeout 300 --timeout-method thread -k "gemm or relu or rope or drelu or fp8 or tight" > gpurun_out/r5_epi_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r5_epi_tests.txt; [ $rc -eq 0 ] || exit $rc
NSTL_LIB_PATH=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd/libnstl_hip_old.so timeout -k 10 200 python tools/bench_gemm_epi.py 2>/dev/null > gpurun_out/r5_epi_old.txt || exit 1
timeout -k 10 200 python tools/bench_gemm_epi.py 2>/dev/null > gpurun_out/r5_epi_new.txt || exit 1
paste gpurun_out/r5_epi_old.txt gpurun_out/r5_epi_new.txt | awk -F'\t' '{print $1 "   |new " substr($2, 24)}'
bash tools/ab_lib.sh 3 "new old"
