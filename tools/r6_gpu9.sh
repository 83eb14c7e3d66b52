#!/bin/bash
# round 6, GPU call 9: the optimizer update overlapped with the next forward (NSTL_ADAM_OVERLAP=1) on the gemm4 kernels: test + step A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_model_gpu.py -k "overlapped" > gpurun_out/r6_g9_tests.txt 2>&1 || { tail -30 gpurun_out/r6_g9_tests.txt; exit 1; }
tail -2 gpurun_out/r6_g9_tests.txt
timeout -k 10 900 bash tools/ab_env.sh NSTL_ADAM_OVERLAP 3 1 0 > gpurun_out/r6_g9_ab.txt 2>&1 || { cat gpurun_out/r6_g9_ab.txt; exit 1; }
cat gpurun_out/r6_g9_ab.txt
NSTL_ADAM_OVERLAP=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6_g9_trace -o run -- python bench.py --steps 3 --warmup 2 --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 > gpurun_out/r6_g9_trace.log 2>&1 || { tail -30 gpurun_out/r6_g9_trace.log; exit 1; }
