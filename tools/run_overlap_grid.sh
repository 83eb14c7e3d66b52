#!/bin/bash
# overlapped optimizer update: step rate vs the update kernel's workgroup cap
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
for rep in 1 2; do
  for cfg in "NSTL_ADAM_OVERLAP=0" "NSTL_ADAM_GRID=32" "NSTL_ADAM_GRID=64" "NSTL_ADAM_GRID=128" "NSTL_ADAM_GRID=512"; do
    env $cfg timeout -k 10 300 python bench.py --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 --steps 30 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['value'], d['ms_per_step'], d['roofline']['achieved'])" || exit 1
  done
done
