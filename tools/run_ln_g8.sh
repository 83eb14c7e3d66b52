#!/bin/bash
# LayerNorm 8-column lane groups: tests, kernel A/B, step A/B
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/ln_ab.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp8_gpu.py tests/test_model_gpu.py > gpurun_out/ln_tests.txt 2>&1 || exit $?
for rep in 1 2; do
  for v in 1 0; do
    echo -n "NSTL_LN_G8=$v " >> gpurun_out/ln_ab.txt
    NSTL_LN_G8=$v timeout -k 10 120 python -u tools/bench_ln.py 2>/dev/null >> gpurun_out/ln_ab.txt || exit $?
  done
done
timeout -k 10 900 bash tools/ab_env.sh NSTL_LN_G8 2 >> gpurun_out/ln_ab.txt 2>&1 || exit $?
