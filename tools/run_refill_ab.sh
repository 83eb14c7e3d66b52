# gemm4 refill after a workgroup's last tile with empty buffer ranges: GEMM GPU tests,
# tools/micro/gemm4_bench G4_EPI_COST=1 (REFILL arms = the live refill, DBG 32768), step A/B
# (old = libnstl_hip_old.so, the previous build)
timeout -k 10 400 python -u -m pytest tests/test_gemm4_gpu.py tests/test_c5_t256_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/refill_gpu_tests.txt 2>&1; tail -1 gpurun_out/refill_gpu_tests.txt
G4_EPI_COST=1 timeout -k 10 200 ./tools/micro/gemm4_bench > gpurun_out/epi_cost5.txt 2>&1 && grep "round 3" gpurun_out/epi_cost5.txt && bash tools/ab_lib.sh 3 > gpurun_out/refill_ab.txt 2>&1; cat gpurun_out/refill_ab.txt
