# the A3/B2 ring (R3) against the two-stage ring on isolated shapes:
# bitwise check, then alternating timings (tools/micro/gemm4_bench.hip, G4_R3_AB)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 env G4_R3_AB=1 tools/micro/gemm4_bench > gpurun_out/${1:-r5}_r3_ab.txt 2>&1 || { tail -20 gpurun_out/${1:-r5}_r3_ab.txt; exit 1; }
cat gpurun_out/${1:-r5}_r3_ab.txt
