# full GPU test suite, bench, and a rocprofv3 kernel-stats profile of 2 warmup + 5 timed steps
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-rX}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -rA > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
cat gpurun_out/${TAG}_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG} -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --no-traffic --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python $GRAFT_REPO_ROOT/tools/prof_summary.py $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}/run_kernel_stats.csv 7 24
timeout -k 10 200 python $GRAFT_REPO_ROOT/tools/bench_gemm_epi.py > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_gemm_epi.txt 2>&1 || exit 1
grep -v amdgpu.ids $GRAFT_REPO_ROOT/gpurun_out/${TAG}_gemm_epi.txt
