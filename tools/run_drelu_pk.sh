# packed dReLU epilogue: GEMM / fp8 / production tests on the new build, the FFN2
# dX shapes old vs new (alternating), then the 228M step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
OLD=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd/libnstl_hip_old.so
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py tests/test_production_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "relu or drelu or gemm or production or fp8" > gpurun_out/drelu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/drelu_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  echo "old: $(NSTL_LIB_PATH=$OLD timeout -k 10 200 python tools/bench_gemm_epi.py 2>/dev/null | grep -E 'DRELU' | tr '\n' ' ')" || exit 1
  echo "new: $(timeout -k 10 200 python tools/bench_gemm_epi.py 2>/dev/null | grep -E 'DRELU' | tr '\n' ' ')" || exit 1
done
bash tools/ab_lib.sh 3
