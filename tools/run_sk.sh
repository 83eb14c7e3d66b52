# stream-K tail: GEMM time against the grid size / CU mask (tools/bench_sk.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/bench_sk.py > gpurun_out/sk_bench.txt 2>&1 || { cat gpurun_out/sk_bench.txt; exit 1; }
cat gpurun_out/sk_bench.txt
