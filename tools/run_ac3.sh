# autocorrelation lag products on f64 MFMA (autocorr3_kernel) vs the register-tiled
# VALU kernel (NSTL_AUTOCORR_V2=1): feature tests, tools/bench_features.py
# alternating (same build, env switch), then a kernel-stats profile of the default
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_features_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ac3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ac3_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for arm in mfma valu; do
    unset NSTL_AUTOCORR_V2
    if [ $arm = valu ]; then export NSTL_AUTOCORR_V2=1; fi
    echo -n "$arm: "; timeout -k 10 120 python tools/bench_features.py 2>/dev/null | tail -1 || exit 1
  done
done
unset NSTL_AUTOCORR_V2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ac3 -o run --output-format csv -- python $R/tools/bench_features.py > $R/gpurun_out/ac3_prof.log 2>&1 || exit 1
python $R/tools/prof_summary.py $R/gpurun_out/prof_ac3/run_kernel_stats.csv 7 10
