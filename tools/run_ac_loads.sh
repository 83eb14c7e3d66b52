# autocorr3 with the frame and window loads in one batch (buffer loads): feature tests, then
# tools/bench_features.py new vs old (HEAD) alternating with one stream
# (NSTL_FEATURES_FORK=0, so the kernels run alone), then kernel stats of both
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_features_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/acl_tests.log 2>&1
rc=$?; tail -1 gpurun_out/acl_tests.log; [ $rc -eq 0 ] || exit $rc
export NSTL_FEATURES_FORK=0
for i in 1 2 3; do
  for arm in new old; do
    unset NSTL_LIB_PATH
    if [ $arm = old ]; then export NSTL_LIB_PATH=$R/neurosync_trainer_lite_amd/libnstl_hip_old.so; fi
    echo -n "$arm: "; timeout -k 10 120 python tools/bench_features.py 2>gpurun_out/acl_$arm.err | tail -1 || { tail -5 gpurun_out/acl_$arm.err; exit 1; }
  done
done
cd /tmp && export TMPDIR=/tmp
for arm in new old; do
  unset NSTL_LIB_PATH
  if [ $arm = old ]; then export NSTL_LIB_PATH=$R/neurosync_trainer_lite_amd/libnstl_hip_old.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_acl_$arm -o run --output-format csv -- python $R/tools/bench_features.py > $R/gpurun_out/acl_prof_$arm.log 2>&1 || exit 1
  echo "$arm:"; python $R/tools/prof_summary.py $R/gpurun_out/prof_acl_$arm/run_kernel_stats.csv 7 3
done
