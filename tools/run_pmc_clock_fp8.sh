# (1) effective clock per kernel family in the bf16 bench (GRBM_GUI_ACTIVE + kernel trace);
# (2) HBM traffic of the fp8 GEMM launches in the --fp8 bench (FETCH_SIZE, WRITE_SIZE passes)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r1_v15}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/pmc_clock -o run --output-format csv -- python $R/bench.py --no-traffic --steps 3 --warmup 2 --no-cpu-baseline --no-parity --feature-steps 0 > $R/gpurun_out/pmc_clock.log 2>&1 || { tail -5 $R/gpurun_out/pmc_clock.log; exit 1; }
python $R/tools/pmc_clock.py $R/gpurun_out/pmc_clock $R/gpurun_out/${TAG}_clock.json $TAG || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch8 -o run --output-format csv -- python $R/bench.py --no-traffic --fp8 --steps 2 --warmup 1 --no-cpu-baseline --no-parity --feature-steps 0 > $R/gpurun_out/pmc_fetch8.log 2>&1 || { tail -5 $R/gpurun_out/pmc_fetch8.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write8 -o run --output-format csv -- python $R/bench.py --no-traffic --fp8 --steps 2 --warmup 1 --no-cpu-baseline --no-parity --feature-steps 0 > $R/gpurun_out/pmc_write8.log 2>&1 || { tail -5 $R/gpurun_out/pmc_write8.log; exit 1; }
python $R/tools/pmc_traffic.py $R/gpurun_out/pmc_fetch8 $R/gpurun_out/pmc_write8 $R/gpurun_out/${TAG}_fp8_gemm_traffic.json ${TAG}_fp8 gemm256f8
