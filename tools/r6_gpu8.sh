#!/bin/bash
# round 6, GPU call 8: fused attention backward with the 49 KB LDS map (3 workgroups per CU): tests, isolated timing, step A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_kernels_gpu.py tests/test_tight_parity_gpu.py tests/test_production_gpu.py > gpurun_out/r6_g8_tests.txt 2>&1 || { tail -30 gpurun_out/r6_g8_tests.txt; exit 1; }
tail -2 gpurun_out/r6_g8_tests.txt
for i in 1 2; do for v in fast full; do echo "NSTL_ATTN_BWD_LDS=$v"; NSTL_ATTN_BWD_LDS=$v timeout -k 10 120 python tools/bench_attn.py 2>&1 | grep -v amdgpu.ids | head -6; done; done > gpurun_out/r6_g8_attn.txt
cat gpurun_out/r6_g8_attn.txt
timeout -k 10 900 bash tools/ab_env.sh NSTL_ATTN_BWD_LDS 3 fast full > gpurun_out/r6_g8_ab.txt 2>&1 || { cat gpurun_out/r6_g8_ab.txt; exit 1; }
cat gpurun_out/r6_g8_ab.txt
