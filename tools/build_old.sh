# Build libnstl_hip.so of git revision $1 (default HEAD) into
# neurosync_trainer_lite_amd/libnstl_hip_old.so (the "old" arm of tools/ab_*.sh).
set -e
REV=${1:-HEAD}
ROOT=$(git rev-parse --show-toplevel)
TMP=$(mktemp -d)
git -C "$ROOT" worktree add -q --detach "$TMP" "$REV"
make -C "$TMP/neurosync_trainer_lite_amd/csrc" -j8 > /dev/null
cp "$TMP/neurosync_trainer_lite_amd/libnstl_hip.so" "$ROOT/neurosync_trainer_lite_amd/libnstl_hip_old.so"
git -C "$ROOT" worktree remove --force "$TMP"
echo "built $REV -> libnstl_hip_old.so"
