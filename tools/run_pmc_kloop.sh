# SQ/TCC counters of the ring GEMM K loop: NN (weight-gradient layout, K = 16384)
# and TN (forward layout, K = 4096), one rocprofv3 --pmc pass per counter group.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-kloop}
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
G2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum"
for shape in "dw 4096 4096 20" "fwd 4096 4096 20"; do
  s=$(echo $shape | tr ' ' '_')
  i=0
  for grp in "$G1" "$G2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp -d $R/gpurun_out/pmc_$TAG/$s/g$i -o run --output-format csv -- python $R/tools/gemm_one.py $shape > $R/gpurun_out/pmc_${TAG}_${s}_g$i.log 2>&1 || { echo "fail $s $i"; tail -5 $R/gpurun_out/pmc_${TAG}_${s}_g$i.log; exit 1; }
  done
  python $R/tools/pmc_gemm_counters.py $R/gpurun_out/pmc_$TAG/$s
done
