#!/bin/bash
# Build libdamvs.so from the sources of a commit: tools/build_at.sh <commit> <out.so>  (A/B and bisection; load it
# with DAMVS_LIB=<out.so>)
set -e
R=$(cd $(dirname $0)/.. && pwd)
C=$1; OUT=$2
T=$(mktemp -d)
git -C $R archive $C damvsnet_amd/csrc include | tar -x -C $T
objs=""
for f in $T/damvsnet_amd/csrc/*.hip $T/damvsnet_amd/csrc/*.cpp; do
  o=$T/$(basename $f).o
  fl=$(python3 -c "import sys; sys.path.insert(0, '$(dirname $0)/..'); from damvsnet_amd.build import FILE_FLAGS; print(' '.join(FILE_FLAGS.get('$(basename "$f")', [])))")   # damvsnet_amd/build.py FILE_FLAGS
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $fl -I$T/include -I$T/damvsnet_amd/csrc -x hip -c $f -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT $objs
rm -rf $T
echo $OUT
