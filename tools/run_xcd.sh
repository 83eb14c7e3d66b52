# grouped-dW XCD remap over the whole launch: tests, step A/B against the
# previous build, the GEMM traffic per family
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm4_gpu.py tests/test_stream_k_gpu.py tests/test_tight_parity_gpu.py -k "grouped or gemm4" -s > gpurun_out/xcd_tests.log 2>&1 || { tail -40 gpurun_out/xcd_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/xcd_tests.log | tail -2
bash tools/ab_lib.sh 2 || exit 1
bash tools/ab_lib.sh 1 "old new" || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 > gpurun_out/xcd_bench.json 2> gpurun_out/xcd_bench.err || { tail -5 gpurun_out/xcd_bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/xcd_bench.json')); r=d['roofline']
print('value', d['value'], 'traffic_vs_alg', r.get('traffic_vs_algorithmic'))
for k,v in r['by_family'].items(): print(k, v['avg_launch_us'], v['frac'], v.get('traffic_vs_algorithmic'))"
