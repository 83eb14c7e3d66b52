# Build a variant of libnstl_hip.so with extra compile flags for one source
# (A/B experiments; the other objects come from the product build):
#   tools/build_variant.sh <tag> <source.hip> <flags...>
#   -> neurosync_trainer_lite_amd/libnstl_hip_<tag>.so
set -e
cd "$(dirname "$0")/../neurosync_trainer_lite_amd/csrc"
TAG=$1; SRC=$2; shift 2
make -s -j8 >/dev/null
mkdir -p build_var/$TAG
base=$(basename $SRC .hip)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function "$@" -c $SRC -o build_var/$TAG/$base.o
objs=""
for o in build/*.o; do
  if [ "$(basename $o)" = "$base.o" ]; then objs="$objs build_var/$TAG/$base.o"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../libnstl_hip_$TAG.so $objs
echo "built libnstl_hip_$TAG.so"
