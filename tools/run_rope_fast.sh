# NSTL_GEMM_ROPE=fast (recomputed RoPE angles in the ring epilogue) against the
# table form: rope tests under the switch, the per-shape epilogue micro-bench in
# both forms, then a same-box step A/B.  tools/run_rope_fast.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
NSTL_GEMM_ROPE=fast timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py tests/test_production_gpu.py -k "rope or production" -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/rope_fast_tests.log 2>&1
rc=$?; tail -3 $O/rope_fast_tests.log; [ $rc -eq 0 ] || exit $rc
for v in table fast table fast; do
  NSTL_GEMM_ROPE=$v timeout -k 10 200 python tools/bench_gemm_epi.py > $O/rope_epi_$v.txt 2>&1 || exit 1
  echo "== $v"; grep -E "ROPE|qkv  BIAS|kvc  BIAS" $O/rope_epi_$v.txt
done
bash tools/ab_env.sh NSTL_GEMM_ROPE 3 table fast
