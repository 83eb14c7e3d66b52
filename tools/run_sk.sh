# stream-K tail + attention epilogue changes: GPU tests, GEMM time against the
# grid size, attention kernel times
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stream_k_gpu.py tests/test_gemm4_gpu.py tests/test_tight_parity_gpu.py -k "not gemm4_production and not ring_f32" tests/test_kernels_gpu.py -s > gpurun_out/sk_tests.log 2>&1 || { tail -40 gpurun_out/sk_tests.log; exit 1; }
grep -E "passed|failed|max \|err\||attention" gpurun_out/sk_tests.log | tail -14
timeout -k 10 200 python tools/bench_sk.py 256 248 240 224 250 > gpurun_out/sk_bench.txt 2>&1 || { cat gpurun_out/sk_bench.txt; exit 1; }
cat gpurun_out/sk_bench.txt
for v in "" "NSTL_BENCH_BIAS=0" "NSTL_BENCH_NOROPE=1"; do echo "--- $v"; env $v timeout -k 10 120 python tools/bench_attn.py 2>/dev/null || exit 1; done
echo "--- CU mask table"
timeout -k 10 400 python tools/cu_mask_bench.py 0 2 4 8 16 --steps 10 --reps 2 > gpurun_out/cu_mask_r4.txt 2>&1 || { tail -5 gpurun_out/cu_mask_r4.txt; exit 1; }
tail -1 gpurun_out/cu_mask_r4.txt
