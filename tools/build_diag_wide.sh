#!/bin/bash
# Diagnostic libdamvs builds of the wide conv2d kernel with parts of its K loop removed (wrong results,
# timing only): damvsnet_amd/ab/libdamvs_wdiag<mask>.so for mask 1 (no MFMA), 2 (no barrier), 4 (no halo
# traffic), 8 (no A loads), 15 (all).
set -e
R=$(cd $(dirname $0)/.. && pwd)
mkdir -p $R/damvsnet_amd/ab
for m in ${@:-1 2 4 8 15}; do
  T=$(mktemp -d)
  objs=""
  for f in $R/damvsnet_amd/csrc/*.hip $R/damvsnet_amd/csrc/*.cpp; do
    o=$T/$(basename $f).o
    fl=$(python3 -c "import sys; sys.path.insert(0, '$(dirname $0)/..'); from damvsnet_amd.build import FILE_FLAGS; print(' '.join(FILE_FLAGS.get('$(basename "$f")', [])))")   # damvsnet_amd/build.py FILE_FLAGS
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $fl ${DIAG_DEFS:--DDAMVS_WIDE_DIAG=$m} -I$R/include -I$R/damvsnet_amd/csrc -x hip -c $f -o $o &
    objs="$objs $o"
  done
  wait
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $R/damvsnet_amd/ab/libdamvs_wdiag$m.so $objs
  rm -rf $T
done
