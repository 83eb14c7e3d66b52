# transposed weight copies for the input-gradient GEMMs (K-major B on the 4-wave kernel): step A/B;
# the CU-mask table with grids sized per (XCD, SE)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stream_k_gpu.py > gpurun_out/wt_tests.log 2>&1 || { tail -30 gpurun_out/wt_tests.log; exit 1; }
tail -1 gpurun_out/wt_tests.log
bash tools/ab_env.sh NSTL_WT 2 1 0 || exit 1
bash tools/ab_env.sh NSTL_WT 1 0 1 || exit 1
echo "--- CU mask table (grids per XCD x SE)"
timeout -k 10 400 python tools/cu_mask_bench.py 0 8 32 64 --steps 10 --reps 2 > gpurun_out/cu_mask_r4c.txt 2>&1 || { tail -5 gpurun_out/cu_mask_r4c.txt; exit 1; }
tail -1 gpurun_out/cu_mask_r4c.txt
