# ReLU-dropout keep bits hashed in the ring GEMM's K loop: tests, FFN1 forward timings, step A/B against the old library
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py tests/test_model_gpu.py tests/test_production_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/keepk_tests.log 2>&1
rc=$?; tail -3 gpurun_out/keepk_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for arm in new old; do
    if [ $arm = old ]; then export NSTL_LIB_PATH=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd/libnstl_hip_old.so; else unset NSTL_LIB_PATH; fi
    timeout -k 10 200 python tools/bench_gemm_epi.py 2>/dev/null | grep -E "ffn1" | grep fwd | sed "s/^/$arm: /" || exit 1
  done
done
unset NSTL_LIB_PATH
bash tools/ab_lib.sh 3
