# T=128: the split attention backward (now two/three workgroups per CU with the
# staging aliased and RoPE^T recomputed) against the fused kernel, 228M step
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_env.sh NSTL_ATTN_BWD 3 fused split
