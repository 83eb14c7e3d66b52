cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/bench_gemm_epi.py > gpurun_out/epi_wt.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/epi_wt.txt | head -20
