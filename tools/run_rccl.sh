# RCCL on one GPU: the collective tests, then the resident-RCCL step cost by
# channel count, then a kernel trace of one probe run (which RCCL kernels run).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_rccl_gpu.py tests/test_dist_gpu.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/rccl_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rccl_tests.log; [ $rc -eq 0 ] || exit $rc
for ch in 1 4 8 16; do
  NCCL_MIN_NCHANNELS=$ch NCCL_MAX_NCHANNELS=$ch timeout -k 10 200 python tools/rccl_probe.py 20 > gpurun_out/rccl_probe_ch$ch.txt 2>&1 || { tail -5 gpurun_out/rccl_probe_ch$ch.txt; exit 1; }
  tail -1 gpurun_out/rccl_probe_ch$ch.txt
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_rccl -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/rccl_probe.py 3 > $GRAFT_REPO_ROOT/gpurun_out/rccl_prof.log 2>&1 || exit 1
grep -i "nccl\|rccl" $GRAFT_REPO_ROOT/gpurun_out/prof_rccl/run_kernel_stats.csv | cut -c1-200 || echo "no RCCL kernel in the trace"
