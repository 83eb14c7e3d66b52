# split attention backward (T=256, BASELINE C5's long clips): parity, kernel times new vs libnstl_hip_old.so
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_model_gpu.py > gpurun_out/t256_tests.log 2>&1 || { tail -40 gpurun_out/t256_tests.log; exit 1; }
tail -2 gpurun_out/t256_tests.log
OLD=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd/libnstl_hip_old.so
for lib in new old; do
  if [ $lib = old ]; then export NSTL_LIB_PATH=$OLD; else unset NSTL_LIB_PATH; fi
  echo "--- $lib T=256"; NSTL_BENCH_T=256 timeout -k 10 120 python tools/bench_attn.py || exit 1
  echo "--- $lib T=128 split"; NSTL_ATTN_BWD=split timeout -k 10 120 python tools/bench_attn.py || exit 1
done
