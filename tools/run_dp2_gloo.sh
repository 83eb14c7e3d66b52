# rehearsal of bench.py's multi-rank path on a 1-GPU box: 2 ranks share cuda:0, gloo collectives
set -o pipefail
cd $GRAFT_REPO_ROOT
NSTL_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --no-traffic --gpus 2 --steps 4 --warmup 2 --feature-steps 0 --batch 32 > gpurun_out/dp2_gloo.json 2> gpurun_out/dp2_gloo.err
rc=$?; tail -3 gpurun_out/dp2_gloo.err; cat gpurun_out/dp2_gloo.json; exit $rc
