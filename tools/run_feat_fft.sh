#!/bin/bash
# fused STFT/mel: feature tests, pipeline A/B (FFT vs DFT GEMM), kernel stats
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_features_gpu.py tests/test_abi.py > gpurun_out/feat_tests.txt 2>&1 || exit $?
for rep in 1 2; do
  for v in 1 0; do
    echo "NSTL_FEATURES_FFT=$v" >> gpurun_out/feat_ab.txt
    NSTL_FEATURES_FFT=$v timeout -k 10 120 python -u tools/bench_features.py >> gpurun_out/feat_ab.txt 2>&1 || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_feat -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/bench_features.py > $GRAFT_REPO_ROOT/gpurun_out/prof_feat.log 2>&1 || exit $?
