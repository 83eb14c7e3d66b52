# concatenated memory-gradient GEMM: model parity (both settings), step A/B by env
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_model_gpu.py > gpurun_out/dmem_tests0.log 2>&1 || { tail -40 gpurun_out/dmem_tests0.log; exit 1; }
tail -1 gpurun_out/dmem_tests0.log
NSTL_DMEM_CONCAT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_model_gpu.py tests/test_dist_gpu.py > gpurun_out/dmem_tests1.log 2>&1 || { tail -40 gpurun_out/dmem_tests1.log; exit 1; }
tail -1 gpurun_out/dmem_tests1.log
bash tools/ab_env.sh NSTL_DMEM_CONCAT 2
