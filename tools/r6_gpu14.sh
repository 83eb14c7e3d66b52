#!/bin/bash
# round 6, GPU call 14: the overlapped update's kernel form (unroll 2 / 4, nontemporal or plain) beside the next forward
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2 3; do
  for arm in "U2NT" "U4NT" "U2PL"; do
    case $arm in U2NT) e="NSTL_ADAM_U=2 NSTL_ADAM_NT=1";; U4NT) e="NSTL_ADAM_U=4 NSTL_ADAM_NT=1";; U2PL) e="NSTL_ADAM_U=2 NSTL_ADAM_NT=0";; esac
    env $e timeout -k 10 300 python bench.py --no-traffic --no-cpu-baseline --no-parity --feature-steps 0 --feed-steps 0 --steps 30 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arm', d['value'], d['ms_per_step'], d['roofline']['achieved'])" || exit 1
  done
done > gpurun_out/r6_g14_adam_form_ab.txt 2>&1
cat gpurun_out/r6_g14_adam_form_ab.txt
