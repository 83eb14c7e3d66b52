#!/bin/bash
# round 6, GPU call 7: ceiling of moving the FFN1 dropout hash out of the epilogue (timing-only build: the hash replaced by one multiply)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 bash tools/ab_libs.sh 4 default neurosync_trainer_lite_amd/libnstl_hip_nohash.so > gpurun_out/r6_g7_nohash_ab.txt 2>&1 || { cat gpurun_out/r6_g7_nohash_ab.txt; tail gpurun_out/ab_libs.err; exit 1; }
cat gpurun_out/r6_g7_nohash_ab.txt
