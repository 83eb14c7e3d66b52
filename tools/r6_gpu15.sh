#!/bin/bash
# round 6, GPU call 15: the GPU suite with the update in order (NSTL_ADAM_OVERLAP=0, the non-default path) and per-layer cross k|v (NSTL_KV_GROUPED=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
NSTL_ADAM_OVERLAP=0 NSTL_KV_GROUPED=0 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_g15_tests_off.txt 2>&1 || { tail -30 gpurun_out/r6_g15_tests_off.txt; exit 1; }
tail -2 gpurun_out/r6_g15_tests_off.txt
