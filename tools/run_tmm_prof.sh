cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_tmm -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/bench_torch_mm.py > $GRAFT_REPO_ROOT/gpurun_out/tmm.log 2>&1 || exit 1
cut -d, -f1-4 $GRAFT_REPO_ROOT/gpurun_out/prof_tmm/run_kernel_stats.csv | head -30
