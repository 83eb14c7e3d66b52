# fp8 tests + micro-bench + same-box A/B (bf16 vs fp8 step, T=128)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-f8}
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_fp8.py > gpurun_out/${TAG}_micro.txt 2>&1 || { tail -5 gpurun_out/${TAG}_micro.txt; exit 1; }
cat gpurun_out/${TAG}_micro.txt
for i in 1 2; do
  for mode in bf16 fp8; do
    flag=""; [ $mode = fp8 ] && flag="--fp8"
    timeout -k 10 200 python bench.py --no-traffic $flag --no-cpu-baseline --no-parity --feature-steps 0 > gpurun_out/${TAG}_${mode}_$i.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_${mode}_$i.json')); print('$mode', $i, d['value'], d['ms_per_step'])"
  done
done
