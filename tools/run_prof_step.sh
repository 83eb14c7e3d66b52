# rocprofv3 kernel-trace summary of the 228M bench step (no counters):
#   tools/run_prof_step.sh <tag> [extra bench args]  ->  gpurun_out/prof_<tag>/ + gpurun_out/<tag>_kernel_stats.csv
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
  python bench.py --steps 20 --warmup 3 --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 "$@" \
  > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
cp $(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1) gpurun_out/${TAG}_kernel_stats.csv
head -30 gpurun_out/${TAG}_kernel_stats.csv | cut -c1-220
