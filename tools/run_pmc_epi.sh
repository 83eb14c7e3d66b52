set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for mode in none skip_store skip_epi; do
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR"; do
    tag=$(echo $grp | cut -d' ' -f1)
    NSTL_GEMM_DEBUG=$mode timeout -k 10 120 rocprofv3 --pmc $grp -d $R/gpurun_out/pmc_epi/$mode/$tag -o run --output-format csv -- python $R/tools/gemm_one.py fwd 4096 256 20 > $R/gpurun_out/pmc_epi_${mode}_$tag.log 2>&1 || { echo "fail $mode $tag"; tail -5 $R/gpurun_out/pmc_epi_${mode}_$tag.log; exit 1; }
  done
done
echo done
