#!/bin/bash
# Build the committed HEAD's libdamvs into damvsnet_amd/ab/libdamvs_base.so (A/B baseline for tools/*bench*).
set -e
R=$(cd $(dirname $0)/.. && pwd)
T=$(mktemp -d)
git -C $R archive HEAD damvsnet_amd/csrc include | tar -x -C $T
mkdir -p $R/damvsnet_amd/ab
objs=""
for f in $T/damvsnet_amd/csrc/*.hip $T/damvsnet_amd/csrc/*.cpp; do
  o=$T/$(basename $f).o
  fl=$(python3 -c "import sys; sys.path.insert(0, '$(dirname $0)/..'); from damvsnet_amd.build import FILE_FLAGS; print(' '.join(FILE_FLAGS.get('$(basename "$f")', [])))")   # damvsnet_amd/build.py FILE_FLAGS
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $fl -I$T/include -I$T/damvsnet_amd/csrc -x hip -c $f -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $R/damvsnet_amd/ab/libdamvs_base.so $objs
rm -rf $T
echo $R/damvsnet_amd/ab/libdamvs_base.so
