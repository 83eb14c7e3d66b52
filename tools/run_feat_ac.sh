#!/bin/bash
# autocorrelation kernel v2: feature tests, pipeline A/B against v1, kernel stats
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/feat_ac_ab.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_features_gpu.py > gpurun_out/feat_ac_tests.txt 2>&1 || exit $?
for rep in 1 2; do
  for v in 0 1; do
    echo "NSTL_AUTOCORR_V1=$v" >> gpurun_out/feat_ac_ab.txt
    NSTL_AUTOCORR_V1=$v timeout -k 10 120 python -u tools/bench_features.py >> gpurun_out/feat_ac_ab.txt 2>&1 || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_feat2 -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/bench_features.py > $GRAFT_REPO_ROOT/gpurun_out/prof_feat2.log 2>&1 || exit $?
