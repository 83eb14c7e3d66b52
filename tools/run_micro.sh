# attention + LayerNorm microbenchmarks (current build)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/bench_attn.py > gpurun_out/attn.txt 2>&1 || exit 1
timeout -k 10 120 python tools/bench_ln.py > gpurun_out/ln.txt 2>&1 || exit 1
cat gpurun_out/attn.txt gpurun_out/ln.txt | grep -v amdgpu
