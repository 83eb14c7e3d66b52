# Adam with U elements per lane and pass (all loads first): bit-identity tests per variant, then the step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
for u in 1 2 4; do
  NSTL_ADAM_U=$u timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k adam -x -q -p no:cacheprovider --timeout 100 --timeout-method thread 2>&1 | tail -1 | sed "s/^/U=$u: /"
done

bash tools/ab_env.sh NSTL_ADAM_U 3 1 2 4
