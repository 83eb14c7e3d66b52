# copy-engine push interference against the number of copy streams (one GPU,
# 8-rank push volume), tools/copy_interference.py --streams k
set -o pipefail
cd $GRAFT_REPO_ROOT
for k in 1 2 3 7; do
  timeout -k 10 300 python tools/copy_interference.py --ranks 8 --streams $k 2>/dev/null | tail -1 || exit 1
done
