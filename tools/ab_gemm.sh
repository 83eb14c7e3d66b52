# GEMM A/B in one box session: kernel tests on the new library, then the
# step's GEMM shapes (tools/bench_gemm_epi.py) alternating old/new builds, then
# the bench step alternating (tools/ab_lib.sh).  old = libnstl_hip_old.so
set -o pipefail
cd $GRAFT_REPO_ROOT
OLD=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd/libnstl_hip_old.so
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_production_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  NSTL_LIB_PATH=$OLD timeout -k 10 200 python tools/bench_gemm_epi.py > gpurun_out/ab_epi_old$i.txt 2>&1 || exit 1
  timeout -k 10 200 python tools/bench_gemm_epi.py > gpurun_out/ab_epi_new$i.txt 2>&1 || exit 1
done
paste gpurun_out/ab_epi_old1.txt gpurun_out/ab_epi_new1.txt gpurun_out/ab_epi_old2.txt gpurun_out/ab_epi_new2.txt | grep -v amdgpu | awk -F'\t' '{printf "%-44s|%-44s|%-44s|%s\n", $1, $2, $3, $4}'
bash tools/ab_lib.sh ${1:-2}
