# round-4 checks: GEMM tests, RoPE epilogue cost, stream-K / masked-stream GEMM
# times, the CU-mask table with the whole-tile default
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm4_gpu.py tests/test_stream_k_gpu.py -s > gpurun_out/sk_tests.log 2>&1 || { tail -40 gpurun_out/sk_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/sk_tests.log | tail -3
timeout -k 10 200 python tools/bench_gemm_epi.py > gpurun_out/epi_r4b.txt 2>&1 || { tail -5 gpurun_out/epi_r4b.txt; exit 1; }
grep -E "qkv|kvc|ffn1" gpurun_out/epi_r4b.txt
timeout -k 10 300 python tools/bench_sk.py > gpurun_out/sk_bench.txt 2>&1 || { cat gpurun_out/sk_bench.txt; exit 1; }
cat gpurun_out/sk_bench.txt
echo "--- CU mask table (stream-K off)"
timeout -k 10 400 python tools/cu_mask_bench.py 0 2 8 16 --steps 10 --reps 2 > gpurun_out/cu_mask_r4b.txt 2>&1 || { tail -5 gpurun_out/cu_mask_r4b.txt; exit 1; }
tail -1 gpurun_out/cu_mask_r4b.txt
