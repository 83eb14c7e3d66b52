# the data-parallel bench path rehearsed on one GPU: 2 ranks, gloo carrying the collectives
# (RCCL refuses two ranks on one device; the driver's 8-GPU run uses RCCL)
set -o pipefail
cd $GRAFT_REPO_ROOT
for mode in zero1_push zero1 zero1_overlap allreduce; do
  NSTL_DP=$mode NSTL_CEDE_CUS=0 NSTL_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-traffic --no-cpu-baseline \
    --no-parity --feature-steps 0 --feed-steps 0 > gpurun_out/dist2_$mode.json 2> gpurun_out/dist2_$mode.err || { tail -20 gpurun_out/dist2_$mode.err; exit 1; }
  echo "$mode: $(cut -c1-300 gpurun_out/dist2_$mode.json)"
done
