# ring kernel (gemm256r) epilogue scratch read by asm: every GPU test, then a step A/B
# (old = libnstl_hip_old.so, the previous build) and the per-kernel profile of the new build
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ring_gpu_tests.txt 2>&1; tail -1 gpurun_out/ring_gpu_tests.txt
bash tools/ab_lib.sh 3 > gpurun_out/ring_ab.txt 2>&1; cat gpurun_out/ring_ab.txt
bash tools/run_prof_step.sh ring_prof > /dev/null 2>&1 && python tools/prof_summary.py gpurun_out/ring_prof_kernel_stats.csv 23 16 2>/dev/null | head -22
