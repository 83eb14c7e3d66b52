# attention A/B in one box session: attention tests on the new library, then
# tools/bench_attn.py alternating old/new builds, then the bench step (ab_lib.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
OLD=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd/libnstl_hip_old.so
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_production_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  NSTL_LIB_PATH=$OLD timeout -k 10 120 python tools/bench_attn.py 2>/dev/null | sed "s/^/old: /" || exit 1
  timeout -k 10 120 python tools/bench_attn.py 2>/dev/null | sed "s/^/new: /" || exit 1
done
bash tools/ab_lib.sh ${1:-2}
