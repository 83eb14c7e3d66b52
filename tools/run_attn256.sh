# split attention backward at T=256 (C5): staging over the operand images (two
# workgroups per CU) and RoPE^T angles recomputed.  Attention / model tests, then
# the C5 bf16 line old (HEAD build) vs new, alternating, and a kernel-stats
# profile of the new build's C5 run
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_production_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "attn or t256 or long or production or rope" > gpurun_out/attn256_tests.log 2>&1
rc=$?; tail -2 gpurun_out/attn256_tests.log; [ $rc -eq 0 ] || exit $rc
C5="--seq 256 --batch 64 --no-traffic --no-cpu-baseline --no-parity --feed-steps 0 --feature-steps 0 --steps 20"
for i in 1 2; do
  for arm in new old; do
    if [ $arm = old ]; then export NSTL_LIB_PATH=$R/neurosync_trainer_lite_amd/libnstl_hip_old.so; else unset NSTL_LIB_PATH; fi
    timeout -k 10 300 python bench.py $C5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm', d['value'], d['ms_per_step'])" || exit 1
  done
done
unset NSTL_LIB_PATH
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_attn256 -o run --output-format csv -- python $R/bench.py $C5 --steps 5 --warmup 2 > $R/gpurun_out/attn256_prof.log 2>&1 || exit 1
python $R/tools/prof_summary.py $R/gpurun_out/prof_attn256/run_kernel_stats.csv 7 14
