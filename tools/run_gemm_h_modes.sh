# gemmh_kernel mode variants (libnstl_hip_hm<m>.so from tools/build_variant.sh):
# GEMM tests on the given variants, then bench_gemm_epi for each, the 256^2
# ring kernel first.  tools/run_gemm_h_modes.sh "<test modes>" "<bench modes>"
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBD=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd
for m in $1; do
  NSTL_GEMM_H=1 NSTL_LIB_PATH=$LIBD/libnstl_hip_hm$m.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py \
    -k "gemm" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/hm${m}_tests.log 2>&1
  rc=$?; echo "hm$m tests: $(tail -1 gpurun_out/hm${m}_tests.log)"; [ $rc -eq 0 ] || exit $rc
done
echo "== ring 256^2"
NSTL_GEMM_H=0 timeout -k 10 200 python tools/bench_gemm_epi.py 2>&1 | grep -v amdgpu.ids || exit 1
for m in $2; do
  echo "== hm$m"
  if [ $m = 0 ]; then unset NSTL_LIB_PATH; else export NSTL_LIB_PATH=$LIBD/libnstl_hip_hm$m.so; fi
  NSTL_GEMM_H=1 timeout -k 10 200 python tools/bench_gemm_epi.py 2>&1 | grep -v amdgpu.ids || exit 1
done
