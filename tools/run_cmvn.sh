# CMVN/delta stage over (coefficient, chunk) and (coefficient, row block) grids:
# feature tests, then tools/bench_features.py new vs old (alternating) and a
# kernel-stats profile of the new build
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_features_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/cmvn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/cmvn_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for arm in new old; do
    unset NSTL_LIB_PATH
    if [ $arm = old ]; then export NSTL_LIB_PATH=$R/neurosync_trainer_lite_amd/libnstl_hip_old.so; fi
    echo -n "$arm: "; timeout -k 10 120 python tools/bench_features.py 2>/dev/null | tail -1 || exit 1
  done
done
unset NSTL_LIB_PATH
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cmvn -o run --output-format csv -- python $R/tools/bench_features.py > $R/gpurun_out/cmvn_prof.log 2>&1 || exit 1
python $R/tools/prof_summary.py $R/gpurun_out/prof_cmvn/run_kernel_stats.csv 7 10
