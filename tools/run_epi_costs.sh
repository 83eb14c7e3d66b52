# epilogue costs on the ring kernel (hipBLASLt off so the plain forms stay native)
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do NSTL_GEMM_LT=0 timeout -k 10 200 python tools/bench_gemm_epi.py 2>/dev/null || exit 1; done
