# loss kernel change: loss / model tests, a kernel trace of the loss kernels, step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_production_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/loss_tests.log 2>&1
rc=$?; tail -3 gpurun_out/loss_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_loss -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --no-traffic --steps 5 --warmup 2 --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/loss_prof.log 2>&1 || exit 1
grep -i "loss" $GRAFT_REPO_ROOT/gpurun_out/prof_loss/run_kernel_stats.csv
cd $GRAFT_REPO_ROOT && bash tools/ab_lib.sh 3
