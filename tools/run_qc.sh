set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/qc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/qc_tests.log; [ $rc -eq 0 ] || exit $rc
for arm in bf16 fp8bwd bf16 fp8bwd; do
  fl=""; [ $arm = fp8bwd ] && fl="--fp8 --fp8-bwd"
  timeout -k 10 300 python bench.py --seq 256 --batch 64 --no-traffic --no-cpu-baseline --feed-steps 0 --feature-steps 0 --no-parity $fl 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm', d['value'], d['ms_per_step'])" || exit 1
done
