# input-gradient GEMMs: LT on W in place (default) vs LT on W^T copies (NSTL_WT=1)
# vs the ring kernel on W^T copies (NSTL_WT=1 NSTL_GEMM_LT=0), 228M step, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
run() {
  env "$@" timeout -k 10 300 python bench.py --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 --steps 30 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['value'], d['ms_per_step'], d['roofline']['achieved'])"
}
for i in 1 2 3; do
  run NSTL_WT=0 || exit 1
  run NSTL_WT=1 || exit 1
  run NSTL_WT=1 NSTL_GEMM_LT=0 || exit 1
done
