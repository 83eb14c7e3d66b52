# fp8 kernel parity tests + fp8 vs bf16 projection timing
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fp8_tests.log 2>&1
rc=$?; tail -25 gpurun_out/fp8_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_fp8.py > gpurun_out/fp8_bench.txt 2>&1 || { tail -5 gpurun_out/fp8_bench.txt; exit 1; }
cat gpurun_out/fp8_bench.txt
