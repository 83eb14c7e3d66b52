# ReLU-dropout keep bits hashed in the K loop.  GEMM tests on
# the new build, then fwd FFN1 + ReLU-dropout old vs new (alternating), then the step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
OLD=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd/libnstl_hip_old.so
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_production_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "relu or drop or gemm or production" > gpurun_out/relu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/relu_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  echo "old: $(NSTL_LIB_PATH=$OLD timeout -k 10 200 python tools/bench_gemm_epi.py 2>/dev/null | grep -E 'ffn1  RELU|fwd ffn1')" || exit 1
  echo "new: $(timeout -k 10 200 python tools/bench_gemm_epi.py 2>/dev/null | grep -E 'ffn1  RELU|fwd ffn1')" || exit 1
done
bash tools/ab_lib.sh 2
