#!/bin/bash
# round 6, GPU call 1: dist tests (IPC/SDMA push + first-step check), the
# self-launcher on a 1-GPU box (refusal, then a gloo rehearsal of 2 ranks), a
# short N=1 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/r6_g1_dist.txt 2>&1 || { echo "dist tests failed"; tail -30 gpurun_out/r6_g1_dist.txt; exit 1; }
tail -3 gpurun_out/r6_g1_dist.txt
timeout -k 10 120 python bench.py --gpus 2 > gpurun_out/r6_g1_refuse.txt 2>&1; echo "refuse rc=$?"; tail -2 gpurun_out/r6_g1_refuse.txt
NSTL_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 4 --warmup 2 --feature-steps 0 --feed-steps 2 --feed-clips 2 --feed-seconds 20 > gpurun_out/r6_g1_gloo2.json 2> gpurun_out/r6_g1_gloo2.err || { echo "gloo rehearsal failed"; tail -30 gpurun_out/r6_g1_gloo2.err; exit 1; }
cat gpurun_out/r6_g1_gloo2.json | head -c 3000
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-traffic --no-cpu-baseline --feature-steps 0 --feed-steps 0 > gpurun_out/r6_g1_bench.json 2> gpurun_out/r6_g1_bench.err || { echo "bench failed"; tail -30 gpurun_out/r6_g1_bench.err; exit 1; }
head -c 600 gpurun_out/r6_g1_bench.json
