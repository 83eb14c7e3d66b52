# round-end evidence on one box: the whole GPU suite, smoke(), the default bench
# line (with its PMC traffic passes and CPU baseline), and a kernel-trace profile
#   tools/run_final.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r5_final}
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
echo "--- C5 (T=256, B=64): bf16 / fp8 forward + FFN2 dX (4-wave fp8 kernel) / the same on the fp8 ring kernel, alternating"
bash tools/run_c5_ab.sh ${TAG} 2 || { echo "c5 failed"; exit 1; }
