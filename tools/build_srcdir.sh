#!/usr/bin/env bash
# Build libdamvs from another source directory (its csrc/ and include/) into damvsnet_amd/ab/libdamvs_<name>.so, for
# A/B runs through DAMVS_LIB of kernels that are not in the working tree (diagnostics).  tools/build_srcdir.sh <name> <dir>
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; S=$2
T=$(mktemp -d)
mkdir -p "$R/damvsnet_amd/ab"
objs=""
for f in "$S"/csrc/*.hip "$S"/csrc/*.cpp; do
  o=$T/$(basename "$f").o
  fl=$(python3 -c "import sys; sys.path.insert(0, '$(dirname $0)/..'); from damvsnet_amd.build import FILE_FLAGS; print(' '.join(FILE_FLAGS.get('$(basename "$f")', [])))")   # damvsnet_amd/build.py FILE_FLAGS
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $fl -I"$S/include" -I"$S/csrc" -x hip -c "$f" -o "$o" &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$R/damvsnet_amd/ab/libdamvs_$name.so" $objs
rm -rf "$T"
echo "$R/damvsnet_amd/ab/libdamvs_$name.so"
