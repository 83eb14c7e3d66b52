set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -k "reduce or step or grad" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/red_tests.log 2>&1
rc=$?; tail -3 gpurun_out/red_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_lib.sh 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_red -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --no-traffic --steps 5 --warmup 2 --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/red_prof.log 2>&1 || exit 1
grep -i "reduce" $GRAFT_REPO_ROOT/gpurun_out/prof_red/run_kernel_stats.csv
