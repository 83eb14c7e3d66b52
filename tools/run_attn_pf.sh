set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pf_tests.log 2>&1
rc=$?; tail -3 gpurun_out/pf_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for m in oneshot persist; do
    NSTL_ATTN_FWD=$m NSTL_BENCH_P=0.3,0.0 timeout -k 10 120 python tools/bench_attn.py 2>/dev/null | sed "s/^/$m: /" || exit 1
  done
done
bash tools/ab_env.sh NSTL_ATTN_FWD 2 persist oneshot
