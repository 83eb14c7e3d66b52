# bench A/B/C... of several builds of the library in one box session (same engine):
#   tools/ab_libs.sh REPS lib_a.so lib_b.so ...   (paths relative to the repo; "default" = the in-tree build)
# arms cycle within each rep so clock drift hits every arm alike
set -o pipefail
cd $GRAFT_REPO_ROOT
REPS=$1; shift
for i in $(seq 1 $REPS); do
  for lib in "$@"; do
    if [ "$lib" = default ]; then unset NSTL_LIB_PATH; else export NSTL_LIB_PATH=$GRAFT_REPO_ROOT/$lib; fi
    timeout -k 10 300 python bench.py --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 --steps 30 2>gpurun_out/ab_libs.err \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['ms_per_step'], d['roofline']['achieved'])" || exit 1
  done
done
