# stft_mel LDS trim (half twiddle table, window read with the samples from global, band bounds in registers: 35 KB, 4 WGs/CU): feature tests, tools/bench_features.py new vs old (HEAD), alternating, then kernel stats of new
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_features_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ac3b_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ac3b_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for arm in new old; do
    unset NSTL_LIB_PATH
    if [ $arm = old ]; then export NSTL_LIB_PATH=$R/neurosync_trainer_lite_amd/libnstl_hip_old.so; fi
    echo -n "$arm: "; timeout -k 10 120 python tools/bench_features.py 2>/dev/null | tail -1 || exit 1
  done
done
unset NSTL_LIB_PATH
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ac3b -o run --output-format csv -- python $R/tools/bench_features.py > $R/gpurun_out/ac3b_prof.log 2>&1 || exit 1
python $R/tools/prof_summary.py $R/gpurun_out/prof_ac3b/run_kernel_stats.csv 7 10
