# bench A/B of one environment switch in one box session:
#   tools/ab_env.sh VAR [reps] [value_a] [value_b]   (default values 1 / 0)
# (alternates VAR=value_a / VAR=value_b runs so clock drift hits both arms alike)
set -o pipefail
cd $GRAFT_REPO_ROOT
VAR=$1; REPS=${2:-2}; VA=${3:-1}; VB=${4:-0}
for i in $(seq 1 $REPS); do
  for v in $VA $VB; do
    env $VAR=$v timeout -k 10 300 python bench.py --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 --steps 30 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$VAR=$v', d['value'], d['ms_per_step'], d['roofline']['achieved'])" || exit 1
  done
done
