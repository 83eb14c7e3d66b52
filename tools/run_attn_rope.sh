# fused attention backward RoPE^T variants: parity, kernel time, step A/B vs libnstl_hip_old.so
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_model_gpu.py > gpurun_out/rope_tests.log 2>&1 || { tail -40 gpurun_out/rope_tests.log; exit 1; }
tail -2 gpurun_out/rope_tests.log
for rb in fast table; do echo "--- rope_bwd=$rb"; NSTL_ROPE_BWD=$rb timeout -k 10 120 python tools/bench_attn.py || exit 1; done
echo "--- norope"; NSTL_BENCH_NOROPE=1 timeout -k 10 120 python tools/bench_attn.py || exit 1
bash tools/ab_lib.sh 2
