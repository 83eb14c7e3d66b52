#!/bin/bash
# round 6, GPU call 16: forward GEMM operand layout, TT vs TN on the step shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_fwd_layout.py > gpurun_out/r6_fwd_layout.txt 2>&1; rc=$?
cat gpurun_out/r6_fwd_layout.txt; exit $rc
