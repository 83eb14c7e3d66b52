# SQ counters of the attention kernels at the 228M step's shape (tools/bench_attn.py),
# one rocprofv3 --pmc pass per counter group.  tools/run_pmc_attn.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
export NSTL_BENCH_P=0.3
R=$GRAFT_REPO_ROOT
TAG=${1:-attn}
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
G2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAVES"
i=0
for grp in "$G1" "$G2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $R/gpurun_out/pmc_$TAG/g$i -o run --output-format csv -- python $R/tools/bench_attn.py > $R/gpurun_out/pmc_${TAG}_g$i.log 2>&1 || { echo "fail $i"; tail -5 $R/gpurun_out/pmc_${TAG}_g$i.log; exit 1; }
done
python $R/tools/pmc_gemm_counters.py $R/gpurun_out/pmc_$TAG attn
