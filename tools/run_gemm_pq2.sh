cd $GRAFT_REPO_ROOT
for i in 1 2; do for v in 0 2; do
  echo "== NSTL_GEMM_PQ=$v"; NSTL_GEMM_PQ=$v timeout -k 10 200 python tools/bench_gemm_epi.py 2>/dev/null | grep -E "fwd ffn1 BIAS|dX  ffn2 bf16|fwd out|fwd ffn2|dX  out" || exit 1
done; done
