#!/bin/bash
# round 6, GPU call 11: self-launched 4-rank rehearsal on one GPU (gloo small collectives, real IPC + SDMA pushes and gathers between 4 processes), B=32 per rank
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
NSTL_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 4 --batch 32 --steps 4 --warmup 2 --feature-steps 0 --feed-steps 0 > gpurun_out/r6_g11_gloo4.json 2> gpurun_out/r6_g11_gloo4.err || { tail -40 gpurun_out/r6_g11_gloo4.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r6_g11_gloo4.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['config'], d['dist'], d['launch'])"
