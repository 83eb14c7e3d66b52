# HBM traffic of the GEMM family in the bench (two separate PMC passes), -> profiles JSON
set -o pipefail
TAG=${1:-r1}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- python $R/bench.py --no-traffic --steps 2 --warmup 1 --no-cpu-baseline --feature-steps 0 > $R/gpurun_out/pmc_fetch.log 2>&1 || { tail -5 $R/gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- python $R/bench.py --no-traffic --steps 2 --warmup 1 --no-cpu-baseline --feature-steps 0 > $R/gpurun_out/pmc_write.log 2>&1 || { tail -5 $R/gpurun_out/pmc_write.log; exit 1; }
python $R/tools/pmc_traffic.py $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write $R/gpurun_out/gemm_traffic.json $TAG
