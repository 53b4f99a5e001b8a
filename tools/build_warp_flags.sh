#!/usr/bin/env bash
# Diagnostic: libdamvs from a source directory with extra compiler flags for k_warp.hip only, into
# damvsnet_amd/ab/libdamvs_<name>.so (DAMVS_LIB A/B).   tools/build_warp_flags.sh <name> <srcdir> <flags...>
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; S=$2; shift 2
T=$(mktemp -d)
mkdir -p "$R/damvsnet_amd/ab"
objs=""
for f in "$S"/csrc/*.hip "$S"/csrc/*.cpp; do
  o=$T/$(basename "$f").o
  extra=""; [ "$(basename "$f")" = k_warp.hip ] && extra="$*"
  fl=$(python3 -c "import sys; sys.path.insert(0, '$(dirname $0)/..'); from damvsnet_amd.build import FILE_FLAGS; print(' '.join(FILE_FLAGS.get('$(basename "$f")', [])))")   # damvsnet_amd/build.py FILE_FLAGS
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $fl -I"$S/include" -I"$S/csrc" $extra -x hip -c "$f" -o "$o" &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$R/damvsnet_amd/ab/libdamvs_$name.so" $objs
rm -rf "$T"
echo "$R/damvsnet_amd/ab/libdamvs_$name.so"
