set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_features_gpu.py -x -q -p no:cacheprovider -k "not c1_train" > gpurun_out/feat_tests.log 2>&1
rc=$?; tail -3 gpurun_out/feat_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python $R/tools/bench_features.py 273.1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_feat -o run --output-format csv -- python $R/tools/bench_features.py 273.1 > $R/gpurun_out/feat_prof.log 2>&1 || exit 1
python $R/tools/prof_summary.py $R/gpurun_out/prof_feat/run_kernel_stats.csv 7 8
