# One recorded version: GPU tests, smoke, bench line, rocprofv3 kernel stats of
# the bench, and the GEMM family's HBM traffic (PMC FETCH_SIZE / WRITE_SIZE in
# separate passes).  tools/run_round.sh <tag>
set -o pipefail
TAG=${1:-rX}
bash $GRAFT_REPO_ROOT/tools/run_bench_prof.sh $TAG || exit 1
bash $GRAFT_REPO_ROOT/tools/run_pmc_traffic.sh $TAG || exit 1
