#!/bin/bash
# GEMM timeline (stamp build) + K-scaling with the epilogue on / skipped / stores skipped
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 240 env NSTL_LIB_PATH=neurosync_trainer_lite_amd/libnstl_hip_stamps.so \
  python -u tools/gemm_timeline.py > gpurun_out/timeline.txt 2>&1 || exit $?
for n in 1024 4096; do
  timeout -k 10 120 python -u tools/bench_gemm_k.py $n > gpurun_out/k_$n.txt 2>&1 || exit $?
  timeout -k 10 120 env NSTL_GEMM_DEBUG=skip_epi python -u tools/bench_gemm_k.py $n > gpurun_out/k_${n}_skipepi.txt 2>&1 || exit $?
  timeout -k 10 120 env NSTL_GEMM_DEBUG=skip_store python -u tools/bench_gemm_k.py $n > gpurun_out/k_${n}_skipstore.txt 2>&1 || exit $?
done
