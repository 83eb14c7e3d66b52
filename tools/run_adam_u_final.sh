# default Adam (U=2): kernel/model/overlap tests, then the step A/B against U=1
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_production_gpu.py tests/test_rccl_gpu.py tests/test_dist_gpu.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/adam_final_tests.log 2>&1
rc=$?; tail -1 gpurun_out/adam_final_tests.log; [ $rc -eq 0 ] || exit $rc
NSTL_ADAM_OVERLAP=1 timeout -k 10 200 python -u -m pytest tests/test_model_gpu.py -k overlap -x -q -p no:cacheprovider --timeout 150 --timeout-method thread 2>&1 | tail -1 || exit 1
bash tools/ab_env.sh NSTL_ADAM_U 3 2 1
