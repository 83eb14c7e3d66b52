# gemmh_kernel (two workgroups per CU) against the 256^2 ring kernel: GEMM
# kernel tests under NSTL_GEMM_H=1, then the epilogue shapes under both.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-h}
NSTL_GEMM_H=${HM:-2} timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 ${HM:-2} 0 ${HM:-2}; do
  echo "== NSTL_GEMM_H=$v"
  NSTL_GEMM_H=$v timeout -k 10 200 python tools/bench_gemm_epi.py 2>&1 | grep -v amdgpu.ids || exit 1
done
