# copy-engine ZeRO-1 on the one-GPU box: the 2-rank bit-identity test (IPC +
# copy engines + nstl_shard_sum), the interference of the pushes' copy-engine
# traffic with the step, and a kernel trace showing no copy kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r5_push}
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_tests.txt
timeout -k 10 400 python tools/copy_interference.py --ranks 8 > gpurun_out/${T}_interference.txt 2>&1 || { tail -20 gpurun_out/${T}_interference.txt; exit 1; }
cat gpurun_out/${T}_interference.txt
timeout -k 10 400 python tools/copy_interference.py --ranks 8 --streams 1 > gpurun_out/${T}_interference_1stream.txt 2>&1 || { tail -20 gpurun_out/${T}_interference_1stream.txt; exit 1; }
tail -1 gpurun_out/${T}_interference_1stream.txt
[ "${2:-}" = "notrace" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${T}_trace -o run -- python3 $GRAFT_REPO_ROOT/tools/copy_interference.py --trace-only > $GRAFT_REPO_ROOT/gpurun_out/${T}_trace.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/${T}_trace.log; exit 1; }
cd $GRAFT_REPO_ROOT
find gpurun_out/${T}_trace -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'echo "copy kernels in the trace:"; grep -ci "copybuffer\|rocclr" {} || true'
find gpurun_out/${T}_trace -name "*memory_copy_stats.csv" | head -1 | xargs -I{} cat {}
