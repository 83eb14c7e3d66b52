# fused clip norm: GPU suite, then step A/B of NSTL_FUSED_NORM (alternating)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/fnorm_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fnorm_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh NSTL_FUSED_NORM 3
