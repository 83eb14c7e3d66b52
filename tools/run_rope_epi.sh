# RoPE GEMM epilogue: positions without a per-row integer modulo.  GEMM tests on
# the new build, then fwd q|k|v + RoPE old vs new (alternating), then the step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
OLD=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd/libnstl_hip_old.so
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "rope or gemm" > gpurun_out/rope_tests.log 2>&1
rc=$?; tail -2 gpurun_out/rope_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  echo "old: $(NSTL_LIB_PATH=$OLD timeout -k 10 200 python tools/bench_gemm_epi.py 2>/dev/null | grep -E 'ROPE')" || exit 1
  echo "new: $(timeout -k 10 200 python tools/bench_gemm_epi.py 2>/dev/null | grep -E 'ROPE')" || exit 1
done
bash tools/ab_lib.sh 2
