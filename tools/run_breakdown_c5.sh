# per-step kernel breakdown of the C5 shape (T=256, B=64), bf16 and fp8+fp8-backward
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for arm in bf16 fp8; do
  fl=""; [ $arm = fp8 ] && fl="--fp8 --fp8-bwd"
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_c5_$arm -o run --output-format csv -- python $R/bench.py --no-traffic --steps 10 --warmup 3 --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 --seq 256 --batch 64 $fl > $R/gpurun_out/c5_$arm.log 2>&1 || exit 1
  echo "== $arm"; python $R/tools/step_breakdown.py $R/gpurun_out/prof_c5_$arm/run_kernel_trace.csv 8 | tee $R/gpurun_out/c5_${arm}_breakdown.txt | head -22
done
