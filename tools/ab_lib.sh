# bench A/B of two builds of the library in one box session (the engine is the
# same): new = libnstl_hip.so, old = libnstl_hip_old.so.  tools/ab_lib.sh [reps] ["old new"]
set -o pipefail
cd $GRAFT_REPO_ROOT
REPS=${1:-2}
ORDER=${2:-new old}  # arm order within a rep (reverse it to check for clock drift)
OLD=$GRAFT_REPO_ROOT/neurosync_trainer_lite_amd/libnstl_hip_old.so
for i in $(seq 1 $REPS); do
  for arm in $ORDER; do
    if [ $arm = old ]; then export NSTL_LIB_PATH=$OLD; else unset NSTL_LIB_PATH; fi
    timeout -k 10 300 python bench.py --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 --steps 30 2>gpurun_out/ab_lib_$arm.err \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm', d['value'], d['ms_per_step'], d['roofline']['achieved'])" || exit 1
  done
done
