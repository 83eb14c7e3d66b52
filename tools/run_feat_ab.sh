# Feature-path GPU tests, then tools/bench_features.py on the new and the old
# library (tools/build_old.sh), alternating, plus a kernel-stats profile of one
# new-library feature run.  tools/run_feat_ab.sh <tag>
set -o pipefail
TAG=${1:-feat}
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_features_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for arm in new old; do
    if [ $arm = old ]; then export NSTL_LIB_PATH=$R/neurosync_trainer_lite_amd/libnstl_hip_old.so; else unset NSTL_LIB_PATH; fi
    echo -n "$arm: "; timeout -k 10 120 python tools/bench_features.py 2>/dev/null | tail -1 || exit 1
  done
done
unset NSTL_LIB_PATH
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG} -o run --output-format csv -- python $R/tools/bench_features.py > $R/gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python $R/tools/prof_summary.py $R/gpurun_out/prof_${TAG}/run_kernel_stats.csv 7 8
cd $R
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -k short_training -x -q -s -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${TAG}_shorttest.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_shorttest.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/short_train_mse.py --steps 300 --out gpurun_out/${TAG}_short_train_mse.json > gpurun_out/${TAG}_short_train.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/${TAG}_short_train.log | tail -5; exit $rc
