# Round-3 session run: new fp8 tests first, then the whole GPU suite, smoke, the
# bench line with its rocprofv3 kernel stats, the C5 lines (bf16 / fp8 forward /
# fp8 forward + backward at T=256, B=64) and the two-rank RCCL probe.
# A failing test does not stop the measurements; a crash, abort or time limit
# (exit 124/134/137/139) stops everything after it.  tools/run_r3.sh <tag>
set -o pipefail
TAG=${1:-r3}
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2: stopping"; exit $1;; esac; }
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/${TAG}_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -v amdgpu.ids $O/${TAG}_$name.log | tail -4
  fatal $rc $name
  return 0
}
step fp8tests 300 python -u -m pytest tests/test_fp8_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -rA -s
step tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rA
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
cat $O/${TAG}_bench.log | grep '^{' > $O/${TAG}_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_${TAG} -o run --output-format csv -- python $R/bench.py --no-traffic --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $R/$O/${TAG}_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; fatal $rc prof
cd $R
python tools/prof_summary.py $O/prof_${TAG}/run_kernel_stats.csv 7 16
for arm in bf16 fp8 fp8bwd; do
  case $arm in bf16) fl="";; fp8) fl="--fp8";; fp8bwd) fl="--fp8 --fp8-bwd";; esac
  step c5_$arm 400 python bench.py --seq 256 --batch 64 --no-traffic --no-cpu-baseline --feed-steps 0 --feature-steps 0 $fl
  grep '^{' $O/${TAG}_c5_$arm.log > $O/${TAG}_c5_$arm.json
done
step rccl2 200 python tools/rccl_2rank_probe.py
# two ranks on the one GPU with gloo carrying the collectives: bench.py's N > 1
# path (ZeRO-1 reduce-scatter / all-gather on device tensors, barriers, the
# max-over-ranks clock, rank 0's line) short of RCCL itself
NSTL_DIST_BACKEND=gloo step dist2_gloo 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0
grep '^{' $O/${TAG}_dist2_gloo.log > $O/${TAG}_dist2_gloo.json
