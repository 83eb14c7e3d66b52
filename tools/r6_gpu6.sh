#!/bin/bash
# round 6, GPU call 6: LayerNorm nontemporal loads / stores (NSTL_LN_NT 1 / 2 / 3): isolated kernels, LN tests, step A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd
for v in default nt1 nt2 nt3; do
  if [ $v = default ]; then unset NSTL_LIB_PATH; else export NSTL_LIB_PATH=$L/libnstl_hip_$v.so; fi
  echo "== $v"; timeout -k 10 200 python tools/bench_mem.py 2>&1 | grep -v amdgpu.ids | head -8 || exit 1
done > gpurun_out/r6_g6_ln_mem.txt 2>&1
cat gpurun_out/r6_g6_ln_mem.txt
NSTL_LIB_PATH=$L/libnstl_hip_nt3.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_kernels_gpu.py tests/test_production_gpu.py > gpurun_out/r6_g6_tests_nt3.txt 2>&1 || { tail -30 gpurun_out/r6_g6_tests_nt3.txt; exit 1; }
tail -2 gpurun_out/r6_g6_tests_nt3.txt
unset NSTL_LIB_PATH
timeout -k 10 900 bash tools/ab_libs.sh 3 default neurosync_trainer_lite_amd/libnstl_hip_nt1.so neurosync_trainer_lite_amd/libnstl_hip_nt2.so neurosync_trainer_lite_amd/libnstl_hip_nt3.so > gpurun_out/r6_g6_nt_ab.txt 2>&1 || { cat gpurun_out/r6_g6_nt_ab.txt; tail gpurun_out/ab_libs.err; exit 1; }
cat gpurun_out/r6_g6_nt_ab.txt
