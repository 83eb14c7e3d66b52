# PMC passes over the feature pipeline: the two autocorrelation kernels
# (autocorr3 = f64 MFMA, default; autocorr2 = register-tiled VALU, NSTL_AUTOCORR_V2=1)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"
for arm in mfma valu; do
  unset NSTL_AUTOCORR_V2
  if [ $arm = valu ]; then export NSTL_AUTOCORR_V2=1; fi
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d $R/gpurun_out/acpmc_${arm}_$i -o run --output-format csv -- python $R/tools/bench_features.py 60 > $R/gpurun_out/acpmc_${arm}_$i.log 2>&1 || exit 1
  done
done
python $R/tools/pmc_kernel.py $R/gpurun_out/acpmc_ autocorr
