# C5 (T = 256, B = 64): kernel traces of the bf16 step and of the fp8 forward +
# fp8 backward step, for a per-launch comparison of the GEMMs fp8 takes over
# (tools/c5_gemm_compare.py).  tools/run_c5_trace.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
C5="--seq 256 --batch 64 --steps 4 --warmup 2 --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0"
i=0
for arm in "" "--fp8 --fp8-bwd"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/c5trace_$i -o run --output-format csv -- \
    python bench.py $C5 $arm > gpurun_out/c5trace_$i.json 2> gpurun_out/c5trace_$i.err || { tail -5 gpurun_out/c5trace_$i.err; exit 1; }
done
python tools/c5_gemm_compare.py gpurun_out/c5trace_1 gpurun_out/c5trace_2
