#!/bin/bash
# round 6, GPU call 10: how many workgroups the overlapped update pieces may use (NSTL_ADAM_GRID) under the next forward
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1100 bash tools/ab_env.sh NSTL_ADAM_GRID 3 8192 2048 1024 512 > gpurun_out/r6_g10_grid_ab.txt 2>&1 || { cat gpurun_out/r6_g10_grid_ab.txt; exit 1; }
cat gpurun_out/r6_g10_grid_ab.txt
