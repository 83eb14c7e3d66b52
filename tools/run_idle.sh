#!/bin/bash
# kernel trace of the resident-input bench step: idle time between kernels
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_idle -o run --output-format csv -- python $R/bench.py --no-traffic --steps 10 --warmup 3 --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 > $R/gpurun_out/prof_idle.log 2>&1 || exit 1
python $R/tools/idle_gaps.py $R/gpurun_out/prof_idle/run_kernel_trace.csv 10
