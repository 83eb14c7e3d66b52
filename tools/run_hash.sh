# cheaper dropout hash: parity/statistics tests, attention / epilogue / LN kernel times, step A/B vs libnstl_hip_old.so
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_model_gpu.py > gpurun_out/hash_tests.log 2>&1 || { tail -40 gpurun_out/hash_tests.log; exit 1; }
tail -2 gpurun_out/hash_tests.log
echo "--- attention new"; timeout -k 10 120 python tools/bench_attn.py || exit 1
echo "--- attention old"; NSTL_LIB_PATH=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd/libnstl_hip_old.so timeout -k 10 120 python tools/bench_attn.py || exit 1
echo "--- ln new"; timeout -k 10 120 python tools/bench_ln.py || exit 1
echo "--- ln old"; NSTL_LIB_PATH=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd/libnstl_hip_old.so timeout -k 10 120 python tools/bench_ln.py || exit 1
echo "--- epi new"; timeout -k 10 200 python tools/bench_gemm_epi.py 2>&1 | grep -E "ffn1|DRELU" || exit 1
echo "--- epi old"; NSTL_LIB_PATH=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd/libnstl_hip_old.so timeout -k 10 200 python tools/bench_gemm_epi.py 2>&1 | grep -E "ffn1|DRELU" || exit 1
bash tools/ab_lib.sh 2
