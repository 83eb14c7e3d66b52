# fused STFT/mel: wave-per-pair kernel (default) vs the workgroup kernel (NSTL_STFT_WG=1): feature tests, tools/bench_features.py
# alternating (same build, env switch), then a kernel-stats profile of the default
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_features_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/stw_tests.log 2>&1
rc=$?; tail -3 gpurun_out/stw_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for arm in wave wg; do
    unset NSTL_STFT_WG
    if [ $arm = wg ]; then export NSTL_STFT_WG=1; fi
    echo -n "$arm: "; timeout -k 10 120 python tools/bench_features.py 2>/dev/null | tail -1 || exit 1
  done
done
unset NSTL_STFT_WG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_stw -o run --output-format csv -- python $R/tools/bench_features.py > $R/gpurun_out/stw_prof.log 2>&1 || exit 1
python $R/tools/prof_summary.py $R/gpurun_out/prof_stw/run_kernel_stats.csv 7 10
