# the GPU suite without -x (every failure in one pass), then smoke() and the bench line
#   tools/run_gpu_tests.sh <tag> [pytest -k expression]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r5}
K=${2:+-k "$2"}
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread $K > gpurun_out/${TAG}_gpu_tests.txt 2>&1
rc=$?
tail -25 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.txt
timeout -k 10 900 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-700 gpurun_out/${TAG}_bench.json
