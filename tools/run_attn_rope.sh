# fused attention backward with LDS-staged RoPE tables: parity, kernel time, step A/B vs libnstl_hip_old.so
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_model_gpu.py > gpurun_out/rope_tests.log 2>&1 || { tail -40 gpurun_out/rope_tests.log; exit 1; }
tail -2 gpurun_out/rope_tests.log
for nr in 0 1; do echo "--- norope=$nr"; NSTL_BENCH_NOROPE=$nr timeout -k 10 120 python tools/bench_attn.py || exit 1; done
bash tools/ab_lib.sh 2
