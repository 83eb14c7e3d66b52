# A/B of the fused-epilogue GEMMs: libnstl_hip_old.so (previous build) vs libnstl_hip.so
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q -p no:cacheprovider > gpurun_out/epi_tests.log 2>&1
rc=$?; tail -3 gpurun_out/epi_tests.log; [ $rc -eq 0 ] || exit $rc
NSTL_LIB_PATH=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd/libnstl_hip_old.so timeout -k 10 200 python tools/bench_gemm_epi.py > gpurun_out/epi_old.txt 2>&1 || exit 1
timeout -k 10 200 python tools/bench_gemm_epi.py > gpurun_out/epi_new.txt 2>&1 || exit 1
paste gpurun_out/epi_old.txt gpurun_out/epi_new.txt | grep -v amdgpu | awk -F'\t' '{printf "%-52s | %s\n", $1, $2}'
