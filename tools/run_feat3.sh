# autocorrelation frame image padded against ds_read_b128 bank conflicts: feature
# GPU tests, tools/bench_features.py new vs old (tools/build_old.sh), alternating,
# and a kernel-stats profile of the new build.  tools/run_feat3.sh <tag>
set -o pipefail
TAG=${1:-feat3}
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_features_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
# arms: old = HEAD build (one workgroup per frame, unpadded image); v2 = this
# build's per-frame kernel (padded image); new = this build's persistent kernel
for i in 1 2 3; do
  for arm in new v2 old; do
    unset NSTL_LIB_PATH NSTL_AUTOCORR_V2
    if [ $arm = old ]; then export NSTL_LIB_PATH=$R/neurosync_trainer_lite_amd/libnstl_hip_old.so; fi
    if [ $arm = v2 ]; then export NSTL_AUTOCORR_V2=1; fi
    echo -n "$arm: "; timeout -k 10 120 python tools/bench_features.py 2>/dev/null | tail -1 || exit 1
  done
done
unset NSTL_LIB_PATH NSTL_AUTOCORR_V2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG} -o run --output-format csv -- python $R/tools/bench_features.py > $R/gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python $R/tools/prof_summary.py $R/gpurun_out/prof_${TAG}/run_kernel_stats.csv 7 8
