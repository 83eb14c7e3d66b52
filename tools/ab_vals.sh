# bench A/B over values of one environment variable in one box session:
#   tools/ab_vals.sh VAR "v1 v2 ..." [reps] [extra bench args]
# (values alternate within each repetition so clock drift hits every arm alike)
set -o pipefail
cd $GRAFT_REPO_ROOT
VAR=$1; VALS=$2; REPS=${3:-2}; shift 3; EXTRA="$@"
for i in $(seq 1 $REPS); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python bench.py --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --steps 30 $EXTRA 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$VAR=$v', d['value'], d['ms_per_step'], d['roofline']['achieved'])" || exit 1
  done
done
