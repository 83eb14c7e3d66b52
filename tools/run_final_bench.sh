# final bench line of the round (default flags: PMC traffic + MFMA-busy passes,
# feature-inclusive and C4 feed legs, parity, CPU baseline) and its rocprofv3
# kernel-stats summary
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r3_v4}
cd $R
timeout -k 10 900 python bench.py > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; grep '^{' gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_bench.json; tail -c 600 gpurun_out/${TAG}_bench.json; echo; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG} -o run --output-format csv -- python $R/bench.py --no-traffic --steps 20 --warmup 5 --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 > $R/gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python $R/tools/prof_summary.py $R/gpurun_out/prof_${TAG}/run_kernel_stats.csv 7 14
