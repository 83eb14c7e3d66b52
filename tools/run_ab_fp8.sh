# same-box A/B of the C5 fp8 step against the bf16 step (T=128), alternating, then a
# rocprof kernel-stats profile of the fp8 step
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-ab8}
for i in 1 2; do
  for mode in bf16 fp8; do
    flag=""; [ $mode = fp8 ] && flag="--fp8"
    timeout -k 10 200 python bench.py --no-traffic $flag --no-cpu-baseline --no-parity --feature-steps 0 > gpurun_out/${TAG}_${mode}_$i.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_${mode}_$i.json')); print('$mode', $i, d['value'], d['ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG} -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --no-traffic --fp8 --steps 5 --warmup 2 --no-cpu-baseline --no-parity --feature-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python $GRAFT_REPO_ROOT/tools/prof_summary.py $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}/run_kernel_stats.csv 7 30
