#!/usr/bin/env bash
# prob_regress rework: regression/stage parity subset, then kbench probreg stage 3 (D=8) and 2 at B=4, A/B vs HEAD.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "${1:-regress or prob or depthnet or forward or stage}" > gpurun_out/pytest_pr.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_pr.log | tail -8
[ $rc -eq 0 ] || exit $rc
for v in "DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_base.so" "DAMVS_X=0"; do
  for s in 3 2; do
    env $v timeout -k 10 120 python tools/kbench.py --kernel probreg --stage $s --batch 4 --iters 20 > gpurun_out/kp.log 2>&1; rc=$?
    echo "$v stage $s: $(grep 'per call' gpurun_out/kp.log)"
    [ $rc -eq 0 ] || { tail -5 gpurun_out/kp.log; exit $rc; }
  done
done
