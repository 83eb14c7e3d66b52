#!/bin/bash
# persistent XCD-phased GEMM: parity tests, timeline, per-shape A/B, step A/B
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 env NSTL_GEMM_PERSIST=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm256" > gpurun_out/persist_tests.txt 2>&1 || exit $?
timeout -k 10 240 env NSTL_LIB_PATH=neurosync_trainer_lite_amd/libnstl_hip_stamps.so \
  python -u tools/gemm_timeline.py > gpurun_out/timeline_persist.txt 2>&1 || exit $?
for rep in 1 2; do
  for arm in "NSTL_GEMM_PERSIST=1" "NSTL_GEMM_PERSIST=0" "NSTL_GEMM_DEBUG=nocut"; do
    echo "== $arm" >> gpurun_out/persist_epi.txt
    timeout -k 10 200 env $arm python -u tools/bench_gemm_epi.py >> gpurun_out/persist_epi.txt 2>&1 || exit $?
  done
done
timeout -k 10 900 bash tools/ab_env.sh NSTL_GEMM_PERSIST 2 > gpurun_out/persist_ab.txt 2>&1 || exit $?
