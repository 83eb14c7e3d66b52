# LDS / MFMA counters of the GEMM kernels in the bf16 bench (one SQ pass)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY -d $R/gpurun_out/pmc_lds -o run --output-format csv -- python $R/bench.py --no-traffic --steps 2 --warmup 1 --no-cpu-baseline --no-parity --feature-steps 0 > $R/gpurun_out/pmc_lds.log 2>&1 || { tail -5 $R/gpurun_out/pmc_lds.log; exit 1; }
python $R/tools/pmc_gemm_counters.py $R/gpurun_out/pmc_lds > $R/gpurun_out/pmc_lds.txt; cat $R/gpurun_out/pmc_lds.txt
