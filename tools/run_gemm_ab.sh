set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider -k "gemm" > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
NSTL_GEMM_RING=0 timeout -k 10 200 python tools/bench_gemm.py > gpurun_out/ab_old.txt 2>&1 || exit 1
timeout -k 10 200 python tools/bench_gemm.py > gpurun_out/ab_new.txt 2>&1 || exit 1
paste gpurun_out/ab_old.txt gpurun_out/ab_new.txt | grep -v amdgpu | awk -F'\t' '{printf "%-55s | %s\n", $1, $2}'
