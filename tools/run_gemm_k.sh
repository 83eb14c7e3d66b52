set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider -k gemm > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_gemm_k.py 4096 0 > gpurun_out/k_new.txt 2>&1 || exit 1
NSTL_GEMM_DEBUG=temporal_store timeout -k 10 200 python tools/bench_gemm_k.py 4096 0 > gpurun_out/k_old.txt 2>&1 || exit 1
paste gpurun_out/k_new.txt gpurun_out/k_old.txt | grep -v amdgpu
