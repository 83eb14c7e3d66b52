# kernel trace of the resident-input bench step only -> per-step breakdown + idle time
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-bd}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python $R/bench.py --no-traffic --steps 10 --warmup 3 --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 > $R/gpurun_out/${TAG}.log 2>&1 || exit 1
python $R/tools/step_breakdown.py $R/gpurun_out/prof_$TAG/run_kernel_trace.csv 8 | tee $R/gpurun_out/${TAG}_breakdown.txt | head -45
