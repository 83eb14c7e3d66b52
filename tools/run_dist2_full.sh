# bench.py's default legs at N = 2 (feature-inclusive and C4 data feed included),
# two ranks on the one GPU with gloo carrying the collectives: the SCALE run's
# code path short of RCCL
set -o pipefail
cd $GRAFT_REPO_ROOT
NSTL_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/dist2_full.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/dist2_full.log | grep -E "^\[bench\]|Traceback|Error" | tail -20; grep '^{' gpurun_out/dist2_full.log > gpurun_out/dist2_full.json; exit $rc
