# C5: fp8 tests, then bench lines alternating bf16 / fp8 at T=256 (B=64, the C5
# long-clip shape) and T=128, each with the parity field (fp8 gated at 1e-3).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-c5}
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for shape in "--seq 256 --batch 64" "--seq 128 --batch 128"; do
  s=$(echo $shape | awk '{print "t"$2}')
  for mode in bf16 fp8 bf16 fp8; do
    flag=""; [ $mode = fp8 ] && flag="--fp8"
    timeout -k 10 300 python bench.py --no-traffic $flag $shape --no-cpu-baseline --feature-steps 0 > gpurun_out/${TAG}_${mode}_$s.json 2> gpurun_out/${TAG}_${mode}_$s.err || { tail -5 gpurun_out/${TAG}_${mode}_$s.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_${mode}_$s.json')); p=d.get('parity',{}); print('$mode', '$s', d['value'], d['ms_per_step'], 'mse_fp8', p.get('mse_fp8'), 'pass', p.get('pass'))"
  done
done
