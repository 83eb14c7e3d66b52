#!/bin/bash
# round 6, GPU call 13: LayerNorm forward with gamma / beta loaded with the row (NSTL_LN_GB_EARLY build): tests, isolated, step A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd
NSTL_LIB_PATH=$L/libnstl_hip_gb.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_kernels_gpu.py tests/test_production_gpu.py > gpurun_out/r6_g13_tests.txt 2>&1 || { tail -30 gpurun_out/r6_g13_tests.txt; exit 1; }
tail -2 gpurun_out/r6_g13_tests.txt
for i in 1 2; do for v in default gb; do
  if [ $v = default ]; then unset NSTL_LIB_PATH; else export NSTL_LIB_PATH=$L/libnstl_hip_gb.so; fi
  echo "== $v"; timeout -k 10 200 python tools/bench_mem.py 2>&1 | grep "LayerNorm fwd" || exit 1
done; done > gpurun_out/r6_g13_mem.txt 2>&1
unset NSTL_LIB_PATH
cat gpurun_out/r6_g13_mem.txt
timeout -k 10 900 bash tools/ab_libs.sh 3 default neurosync_trainer_lite_amd/libnstl_hip_gb.so > gpurun_out/r6_g13_ab.txt 2>&1 || { cat gpurun_out/r6_g13_ab.txt; exit 1; }
cat gpurun_out/r6_g13_ab.txt
