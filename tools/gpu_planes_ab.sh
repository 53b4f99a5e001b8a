#!/usr/bin/env bash
# conv2d_planes A/B: front-end parity, then kbench2d plane-only layers for the HEAD build
# (ab/libdamvs_base.so) and the working tree.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontend.py -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_fe.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_fe.log
[ $rc -eq 0 ] || exit $rc
for v in "DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_base.so" ${EXTRA:-} "DAMVS_NONE=1"; do
  echo "== $v"
  env $v timeout -k 10 120 python -u tools/kbench2d.py --only ${ONLY:-W,X,Y} > gpurun_out/kb.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/kb.log | grep -v copy
  [ $rc -eq 0 ] || exit $rc
done
