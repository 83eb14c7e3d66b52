#!/bin/bash
# round 6, GPU call 3: C5 T=256 test (4-wave fp8 route assertion), a kernel trace of a short bench (where the copy kernels come from)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_c5_t256_gpu.py > gpurun_out/r6_g3_c5.txt 2>&1 || { tail -30 gpurun_out/r6_g3_c5.txt; exit 1; }
tail -3 gpurun_out/r6_g3_c5.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r6_g3_trace -o run -- python bench.py --steps 3 --warmup 2 --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 > gpurun_out/r6_g3_trace.log 2>&1 || { tail -30 gpurun_out/r6_g3_trace.log; exit 1; }
find gpurun_out/r6_g3_trace -name "*.csv" | head
timeout -k 10 120 tools/micro/hbm_rate > gpurun_out/r6_g3_hbm_rate.txt 2>&1 || { tail -5 gpurun_out/r6_g3_hbm_rate.txt; exit 1; }
cat gpurun_out/r6_g3_hbm_rate.txt
