# round-end evidence on one box: the whole GPU suite, smoke(), the default bench
# line (with its PMC traffic passes and CPU baseline), and a kernel-trace profile
#   tools/run_final.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r4_final}
if [ "${2:-all}" != "prof" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.txt
timeout -k 10 900 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json | cut -c1-600
fi
[ "${2:-all}" = "tests" ] && exit 0
bash tools/run_prof_step.sh ${TAG}_prof > /dev/null 2>&1 || { echo "profile failed"; exit 1; }
python tools/prof_summary.py gpurun_out/${TAG}_prof_kernel_stats.csv 23 16 2>/dev/null | head -30
echo "--- C5 (T=256, B=64): bf16 / fp8 forward / fp8 forward + backward, alternating"
C5="--seq 256 --batch 64 --steps 15 --warmup 3 --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0"
for rep in 1 2; do
  for arm in "" "--fp8" "--fp8 --fp8-bwd"; do
    timeout -k 10 300 python bench.py $C5 $arm > gpurun_out/${TAG}_c5.json 2>/dev/null || { echo "c5 $arm failed"; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_c5.json')); print('c5 %-16s %.1f frames/s %.2f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$arm" | tee -a gpurun_out/${TAG}_c5_ab.txt
  done
done
