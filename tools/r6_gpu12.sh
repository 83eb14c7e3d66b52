#!/bin/bash
# round 6, GPU call 12: the step on a high-priority stream (side streams at default priority): A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
NSTL_HIPRIO=1 timeout -k 10 200 python bench.py --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 --steps 5 2>&1 | grep -E "priority|value" | cut -c1-200
timeout -k 10 900 bash tools/ab_env.sh NSTL_HIPRIO 3 1 0 > gpurun_out/r6_g12_prio_ab.txt 2>&1 || { cat gpurun_out/r6_g12_prio_ab.txt; exit 1; }
cat gpurun_out/r6_g12_prio_ab.txt
