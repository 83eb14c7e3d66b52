#!/bin/bash
# round 6, GPU call 2: the whole zero1_push exchange at the 8-rank volume on one GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python tools/copy_interference.py --exchange --ranks 8 --steps 20 --reps 3 > gpurun_out/r6_g2_exchange8.txt 2> gpurun_out/r6_g2_exchange8.err || { tail -20 gpurun_out/r6_g2_exchange8.err; exit 1; }
cat gpurun_out/r6_g2_exchange8.txt
timeout -k 10 400 python tools/copy_interference.py --exchange --ranks 2 --steps 20 --reps 2 > gpurun_out/r6_g2_exchange2.txt 2> gpurun_out/r6_g2_exchange2.err || { tail -20 gpurun_out/r6_g2_exchange2.err; exit 1; }
cat gpurun_out/r6_g2_exchange2.txt
