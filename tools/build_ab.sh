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
  fl=""; [ "$(basename $f)" = k_warp.hip ] && fl="-fno-slp-vectorize"   # as damvsnet_amd/build.py FILE_FLAGS
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $fl -I$T/include -I$T/damvsnet_amd/csrc -x hip -c $f -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $R/damvsnet_amd/ab/libdamvs_base.so $objs
rm -rf $T
echo $R/damvsnet_amd/ab/libdamvs_base.so
