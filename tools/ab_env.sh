# bench A/B(/C...) of one environment switch in one box session:
#   tools/ab_env.sh VAR [reps] [value ...]   (default values 1 0)
# (cycles through the values each rep so clock drift hits every arm alike)
set -o pipefail
cd $GRAFT_REPO_ROOT
VAR=$1; REPS=${2:-2}; shift; shift
VALS=${@:-1 0}
for i in $(seq 1 $REPS); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python bench.py --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 --steps 30 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$VAR=$v', d['value'], d['ms_per_step'], d['roofline']['achieved'])" || exit 1
  done
done
