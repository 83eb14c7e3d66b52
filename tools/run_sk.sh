# round-4 checks: stream-K tail (XCD-contiguous ranks), GPU tests, GEMM time
# against the grid size, the CU-mask table
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attn_persist_gpu.py tests/test_stream_k_gpu.py tests/test_gemm4_gpu.py -s > gpurun_out/sk_tests.log 2>&1 || { tail -40 gpurun_out/sk_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/sk_tests.log | tail -3
timeout -k 10 200 python tools/bench_sk.py 256 248 240 224 > gpurun_out/sk_bench.txt 2>&1 || { cat gpurun_out/sk_bench.txt; exit 1; }
cat gpurun_out/sk_bench.txt
echo "--- CU mask table"
timeout -k 10 400 python tools/cu_mask_bench.py 0 2 4 8 16 --steps 10 --reps 2 > gpurun_out/cu_mask_r4.txt 2>&1 || { tail -5 gpurun_out/cu_mask_r4.txt; exit 1; }
tail -1 gpurun_out/cu_mask_r4.txt
