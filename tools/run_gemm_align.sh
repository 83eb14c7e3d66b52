# GEMM tests after the epilogue's C-alignment check (vector stores only on aligned
# C), then a quick same-box step A/B against HEAD (the check is a scalar compare)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/align_tests.log 2>&1
rc=$?; tail -3 gpurun_out/align_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_lib.sh 2
