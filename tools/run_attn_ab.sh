# attention kernel tests + fused vs split backward timing at the 228M shape
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k attention -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -15 gpurun_out/attn_tests.log; [ $rc -eq 0 ] || exit $rc
NSTL_ATTN_BWD=split timeout -k 10 120 python tools/bench_attn.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 python tools/bench_attn.py 2>&1 | grep -v amdgpu.ids
