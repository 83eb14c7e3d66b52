# effective clock + MFMA busy per kernel over a 1+2-step bench run (one PMC pass)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d $R/gpurun_out/pmc_clock -o run --output-format csv -- python $R/bench.py --no-traffic --steps 2 --warmup 1 --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 > $R/gpurun_out/pmc_clock.log 2>&1 || { tail -5 $R/gpurun_out/pmc_clock.log; exit 1; }
python $R/tools/pmc_clock.py $R/gpurun_out/pmc_clock 2
