# fp8 4-wave kernel with epilogue side data (scales + bias / keep-bit words by LDS-DMA):
# the fp8 / C5 / GEMM GPU tests, then C5 fp8 step A/B against libnstl_hip_old.so (the previous build)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_fp8_gpu.py tests/test_c5_t256_gpu.py tests/test_gemm4_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/f8side_tests.txt 2>&1 || { tail -30 gpurun_out/f8side_tests.txt; exit 1; }
tail -1 gpurun_out/f8side_tests.txt
C5="--seq 256 --batch 64 --steps 15 --warmup 3 --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 --fp8 --fp8-bwd"
for rep in 1 2 3; do
  for arm in new old; do
    if [ $arm = old ]; then export NSTL_LIB_PATH=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd/libnstl_hip_old.so; else unset NSTL_LIB_PATH; fi
    timeout -k 10 300 python bench.py $C5 > gpurun_out/f8side_c5.json 2>gpurun_out/f8side_c5.err || { tail -20 gpurun_out/f8side_c5.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/f8side_c5.json')); print('c5 fp8 %-4s %.1f frames/s %.2f ms' % (sys.argv[1], d['value'], d['ms_per_step']))" "$arm"
  done
done
