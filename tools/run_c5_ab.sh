# C5 (T = 256, B = 64) step A/B: bf16, fp8 forward + FFN2 dX on the 4-wave fp8
# kernel (default), and the same on the fp8 ring kernel (NSTL_GEMM4_F8=0);
# alternating arms, REPS rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r5_c5}; REPS=${2:-2}
C5="--seq 256 --batch 64 --steps 15 --warmup 3 --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0"
for rep in $(seq 1 $REPS); do
  for arm in "bf16" "fp8" "fp8ring"; do
    case $arm in
      bf16) ARGS=""; ENVV="NSTL_GEMM4_F8=1";;
      fp8) ARGS="--fp8 --fp8-bwd"; ENVV="NSTL_GEMM4_F8=1";;
      fp8ring) ARGS="--fp8 --fp8-bwd"; ENVV="NSTL_GEMM4_F8=0";;
    esac
    env $ENVV timeout -k 10 300 python bench.py $C5 $ARGS > gpurun_out/${TAG}_c5.json 2>gpurun_out/${TAG}_c5.err || { tail -20 gpurun_out/${TAG}_c5.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_c5.json')); print('c5 %-8s %.1f frames/s %.2f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$arm" | tee -a gpurun_out/${TAG}_c5_ab.txt
  done
done
