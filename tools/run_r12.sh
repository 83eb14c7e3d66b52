set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/r12_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/r12_tests.log; tail -5 gpurun_out/r12_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-traffic > gpurun_out/r12_bench.json 2> gpurun_out/r12_bench.err
rc=$?; cat gpurun_out/r12_bench.json; exit $rc
