# attention kernels: their GPU tests on the new library, then tools/bench_attn.py
# alternating the old (libnstl_hip_old.so) and new builds.  tools/run_attn_ab.sh [reps]
set -o pipefail
cd $GRAFT_REPO_ROOT
OLD=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd/libnstl_hip_old.so
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attn or attention or dropout" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/attn_ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/attn_ab_tests.log; [ $rc -eq 0 ] || exit $rc
for i in $(seq ${1:-3}); do
  NSTL_LIB_PATH=$OLD timeout -k 10 120 python tools/bench_attn.py 2>/dev/null | sed "s/^/old: /" || exit 1
  timeout -k 10 120 python tools/bench_attn.py 2>/dev/null | sed "s/^/new: /" || exit 1
done
