#!/usr/bin/env bash
# Warp kernel A/B: parity subset, then kbench warp stages 1-3 at B=4 for the HEAD build (ab/libdamvs_base.so,
# tools/build_ab.sh), the working tree, and the working tree without the view pipeline.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "${1:-warp or stage or sharded or odd_batch}" > gpurun_out/pytest_warp.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_warp.log | tail -8
[ $rc -eq 0 ] || exit $rc
for v in "DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_base.so" "DAMVS_WARP_NO_PIPE=0" "DAMVS_WARP_NO_PIPE=1"; do
  for s in 1 2 3; do
    env $v timeout -k 10 120 python tools/kbench.py --kernel warp --stage $s --batch 4 --iters 20 > gpurun_out/kw.log 2>&1; rc=$?
    echo "$v stage $s: $(grep 'per call' gpurun_out/kw.log)"
    [ $rc -eq 0 ] || { tail -5 gpurun_out/kw.log; exit $rc; }
  done
done
