# HBM bytes of the attention kernels at the 228M step's shape (tools/bench_attn.py, p = 0.3):
# rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes, per-dispatch means (KiB).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export NSTL_BENCH_P=0.3
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c -d $R/gpurun_out/attn_traffic/$c -o run --output-format csv -- python $R/tools/bench_attn.py > $R/gpurun_out/attn_traffic_$c.log 2>&1 || { echo "fail $c"; tail -5 $R/gpurun_out/attn_traffic_$c.log; exit 1; }
done
python $R/tools/pmc_kernel.py $R/gpurun_out/attn_traffic/ attn_
