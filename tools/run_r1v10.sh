# epilogue isolation microbench + GEMM HBM traffic (PMC) of the current tree
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/bench_gemm_epi.py > gpurun_out/epi_v10.txt 2>&1 || { tail -5 gpurun_out/epi_v10.txt; exit 1; }
cat gpurun_out/epi_v10.txt
bash tools/run_pmc_traffic.sh r1_v10
