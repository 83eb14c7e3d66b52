# feature pipeline: autocorrelation forked onto a side stream (default) vs one stream (NSTL_FEATURES_FORK=0): feature tests,
# tools/bench_features.py alternating (same build, env switch), then a kernel trace of the default
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_features_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/fork_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fork_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for arm in fork one; do
    unset NSTL_FEATURES_FORK
    if [ $arm = one ]; then export NSTL_FEATURES_FORK=0; fi
    echo -n "$arm: "; timeout -k 10 120 python tools/bench_features.py 2>/dev/null | tail -1 || exit 1
  done
done
unset NSTL_FEATURES_FORK
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_fork -o run --output-format csv -- python $R/tools/bench_features.py > $R/gpurun_out/fork_prof.log 2>&1 || exit 1
python $R/tools/prof_summary.py $R/gpurun_out/prof_fork/run_kernel_stats.csv 7 10
