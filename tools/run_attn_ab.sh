# attention kernels: parity tests, kernel times new vs libnstl_hip_old.so, step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_model_gpu.py > gpurun_out/attn_tests.log 2>&1 || { tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
echo "--- attention new"; timeout -k 10 120 python tools/bench_attn.py || exit 1
echo "--- attention old"; NSTL_LIB_PATH=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd/libnstl_hip_old.so timeout -k 10 120 python tools/bench_attn.py || exit 1
bash tools/ab_lib.sh ${1:-2}
