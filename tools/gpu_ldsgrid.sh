#!/usr/bin/env bash
# A/B of the persistent conv2d_lds grid size (DAMVS_CONV2D_LDS_GRID; 0 = one block per tile) on the
# thin full-resolution layers, then the front-end parity tests.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
for G in ${GRIDS:-0 1024 2048 4096}; do
  echo "== grid $G"
  DAMVS_CONV2D_LDS_GRID=$G timeout -k 10 120 python -u tools/kbench2d.py --only ${ONLY:-A,C,P,U,V} > gpurun_out/ldsgrid_$G.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/ldsgrid_$G.log
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontend.py -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_fe.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_fe.log
exit $rc
