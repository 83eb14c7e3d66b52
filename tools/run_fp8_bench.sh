# fp8 tests, then C5-style bench lines: fp8 at T=128 and T=256, bf16 at T=256 for comparison
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/fp8_tests.log 2>&1
rc=$?; tail -4 gpurun_out/fp8_tests.log; [ $rc -eq 0 ] || exit $rc
TAG=${1:-fp8}
timeout -k 10 300 python bench.py --no-traffic --fp8 --no-cpu-baseline --feature-steps 0 > gpurun_out/${TAG}_c5_t128.json 2> gpurun_out/${TAG}_c5_t128.err || { tail -5 gpurun_out/${TAG}_c5_t128.err; exit 1; }
cat gpurun_out/${TAG}_c5_t128.json
timeout -k 10 300 python bench.py --no-traffic --fp8 --seq 256 --batch 64 --no-cpu-baseline --feature-steps 0 > gpurun_out/${TAG}_c5_t256.json 2> gpurun_out/${TAG}_c5_t256.err || { tail -5 gpurun_out/${TAG}_c5_t256.err; exit 1; }
cat gpurun_out/${TAG}_c5_t256.json
timeout -k 10 300 python bench.py --no-traffic --seq 256 --batch 64 --no-cpu-baseline --feature-steps 0 --no-parity > gpurun_out/${TAG}_bf16_t256.json 2> gpurun_out/${TAG}_bf16_t256.err || { tail -5 gpurun_out/${TAG}_bf16_t256.err; exit 1; }
cat gpurun_out/${TAG}_bf16_t256.json
