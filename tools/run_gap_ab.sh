# host-side step overhead: model tests, then bench new vs old (HEAD) alternating
# (both python trees: the old arm runs _abtree/, a git archive of HEAD), then
# a kernel trace of the new build and its per-step GPU idle (tools/gap_check.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_production_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gap_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gap_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for arm in new old; do
    if [ $arm = new ]; then d=$R; else d=$R/_abtree; fi
    (cd $d && timeout -k 10 300 python bench.py --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 --steps 30 2>/dev/null) \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm', d['value'], d['ms_per_step'])" || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_gap -o run --output-format csv -- python $R/bench.py --no-traffic --steps 12 --warmup 3 --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 > $R/gpurun_out/gap_prof.log 2>&1 || exit 1
python $R/tools/gap_check.py $R/gpurun_out/prof_gap
