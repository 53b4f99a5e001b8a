#!/usr/bin/env bash
# Build the working tree's libdamvs with extra compiler flags into damvsnet_amd/ab/libdamvs_<name>.so, for A/B
# runs through DAMVS_LIB (e.g. tools/build_variant.sh noocc -DDAMVS_NO_OCC).
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
T=$(mktemp -d)
mkdir -p "$R/damvsnet_amd/ab"
objs=""
for f in "$R"/damvsnet_amd/csrc/*.hip "$R"/damvsnet_amd/csrc/*.cpp; do
  o=$T/$(basename "$f").o
  fl=$(python3 -c "import sys; sys.path.insert(0, '$(dirname $0)/..'); from damvsnet_amd.build import FILE_FLAGS; print(' '.join(FILE_FLAGS.get('$(basename "$f")', [])))")   # damvsnet_amd/build.py FILE_FLAGS
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $fl -I"$R/include" -I"$R/damvsnet_amd/csrc" "$@" -x hip -c "$f" -o "$o" &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$R/damvsnet_amd/ab/libdamvs_$name.so" $objs
rm -rf "$T"
echo "$R/damvsnet_amd/ab/libdamvs_$name.so"
