#!/bin/bash
# round 6, GPU call 5: GEMM epilogue store cache policy (plain / sc1 write-through / nt; + LN and attention-forward sc1): correctness of the variants, step A/B, kernel traces
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in pol1 pol1all; do
NSTL_LIB_PATH=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd/libnstl_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gemm4_gpu.py tests/test_production_gpu.py > gpurun_out/r6_g5_tests_$v.txt 2>&1 || { tail -30 gpurun_out/r6_g5_tests_$v.txt; exit 1; }
tail -2 gpurun_out/r6_g5_tests_$v.txt
done
timeout -k 10 900 bash tools/ab_libs.sh 3 default neurosync_trainer_lite_amd/libnstl_hip_pol1.so neurosync_trainer_lite_amd/libnstl_hip_pol2.so neurosync_trainer_lite_amd/libnstl_hip_pol1all.so > gpurun_out/r6_g5_pol_ab.txt 2>&1 || { cat gpurun_out/r6_g5_pol_ab.txt; tail gpurun_out/ab_libs.err; exit 1; }
cat gpurun_out/r6_g5_pol_ab.txt
for v in pol1 pol1all; do
NSTL_LIB_PATH=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd/libnstl_hip_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6_g5_trace_$v -o run -- python bench.py --steps 3 --warmup 2 --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 > gpurun_out/r6_g5_trace_$v.log 2>&1 || { tail -30 gpurun_out/r6_g5_trace_$v.log; exit 1; }
done
