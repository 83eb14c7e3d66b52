#!/bin/bash
# round 6, GPU call 4: grouped cross k|v RoPE GEMM (test + production parity tests + step A/B), C5 test, kernel trace, HBM rates
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gemm4_gpu.py tests/test_production_gpu.py tests/test_c5_t256_gpu.py > gpurun_out/r6_g4_tests.txt 2>&1 || { tail -40 gpurun_out/r6_g4_tests.txt; exit 1; }
tail -3 gpurun_out/r6_g4_tests.txt
timeout -k 10 600 bash tools/ab_env.sh NSTL_KV_GROUPED 3 1 0 > gpurun_out/r6_g4_kv_ab.txt 2>&1 || { cat gpurun_out/r6_g4_kv_ab.txt; exit 1; }
cat gpurun_out/r6_g4_kv_ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r6_g4_trace -o run -- python bench.py --steps 3 --warmup 2 --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 > gpurun_out/r6_g4_trace.log 2>&1 || { tail -30 gpurun_out/r6_g4_trace.log; exit 1; }
timeout -k 10 120 tools/micro/hbm_rate > gpurun_out/r6_g4_hbm_rate.txt 2>&1 || { tail -5 gpurun_out/r6_g4_hbm_rate.txt; exit 1; }
cat gpurun_out/r6_g4_hbm_rate.txt
