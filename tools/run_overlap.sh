#!/bin/bash
# optimizer update overlapped with the next forward: equivalence tests + step A/B
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_model_gpu.py tests/test_abi.py > gpurun_out/overlap_tests.txt 2>&1 || exit $?
timeout -k 10 900 bash tools/ab_env.sh NSTL_ADAM_OVERLAP 3 > gpurun_out/overlap_ab.txt 2>&1 || exit $?
