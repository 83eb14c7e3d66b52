# Round-end C5 record on HEAD: bf16 / fp8 forward / fp8 forward + backward at
# T=256, B=64, two passes in alternating order (same box), then bench.py's N=2
# path with gloo on the one GPU.  tools/run_c5_final.sh <tag>
set -o pipefail
TAG=${1:-c5f}
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
for rep in 1 2; do
  for arm in bf16 fp8 fp8bwd; do
    case $arm in bf16) fl="";; fp8) fl="--fp8";; fp8bwd) fl="--fp8 --fp8-bwd";; esac
    timeout -k 10 400 python bench.py --seq 256 --batch 64 --no-traffic --no-cpu-baseline --feed-steps 0 --feature-steps 0 $fl > $O/${TAG}_c5_${arm}_$rep.log 2>&1 || { tail -5 $O/${TAG}_c5_${arm}_$rep.log; exit 1; }
    grep '^{' $O/${TAG}_c5_${arm}_$rep.log > $O/${TAG}_c5_${arm}_$rep.json
    python -c "import json; d=json.load(open('$O/${TAG}_c5_${arm}_$rep.json')); p=d.get('parity',{}); print('$arm', $rep, d['value'], d['ms_per_step'], 'mse_fp8', p.get('mse_fp8'), 'pass_fp8', p.get('pass_fp8'))"
  done
done
NSTL_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 > $O/${TAG}_dist2_gloo.log 2>&1 || { tail -5 $O/${TAG}_dist2_gloo.log; exit 1; }
grep '^{' $O/${TAG}_dist2_gloo.log > $O/${TAG}_dist2_gloo.json
cat $O/${TAG}_dist2_gloo.json
