timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/side_gpu_tests.txt 2>&1; tail -2 gpurun_out/side_gpu_tests.txt
G4_EPI_COST=1 timeout -k 10 200 ./tools/micro/gemm4_bench > gpurun_out/epi_cost4.txt 2>&1 && grep "round 3" gpurun_out/epi_cost4.txt && bash tools/ab_lib.sh 3 > gpurun_out/side_ab.txt 2>&1; cat gpurun_out/side_ab.txt
