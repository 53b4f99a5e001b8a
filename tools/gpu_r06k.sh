#!/bin/bash
# Round-6 A/B: wide-kernel N-group skip (product) against -DDAMVS_WIDE_NG_SKIP=0 (damvsnet_amd/ab/libdamvs_ngoff.so):
# front-end GPU tests, kbench2d both dtypes both builds, then the bench line of each build.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06k}
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_frontend.py > gpurun_out/r06/${T}_pytest_frontend.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r06/${T}_pytest_frontend.log; [ $rc -eq 0 ] || exit $rc
for dt in f32 bf16; do
  timeout -k 10 200 python -u tools/kbench2d.py --dtype $dt > gpurun_out/r06/${T}_k2d_${dt}_skip.txt 2>&1 || exit 7
  DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_ngoff.so timeout -k 10 200 python -u tools/kbench2d.py --dtype $dt > gpurun_out/r06/${T}_k2d_${dt}_off.txt 2>&1 || exit 7
  paste gpurun_out/r06/${T}_k2d_${dt}_skip.txt gpurun_out/r06/${T}_k2d_${dt}_off.txt | grep " us" | awk -F'\t' '{print $1 " || " $2}' | cut -c1-160
done
TAG=${T} bash tools/gpu_ab.sh "skip|DAMVS_X=1|" "off|DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_ngoff.so|" "skip2|DAMVS_X=1|" "off2|DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_ngoff.so|"
