#!/bin/bash
# Quick GPU iteration: parity subset (-k expression $1, default all gpu tests) + hot-path kernel microbench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
K=${1:-""}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider ${K:+-k "$K"} > gpurun_out/pytest_q.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|Error" gpurun_out/pytest_q.log | tail -15
[ $rc -le 1 ] || exit $rc
shift; [ $# -gt 0 ] || set -- "warp 1" "warp 2" "warp 3"
for k in "$@"; do set -- $k; timeout -k 10 120 python tools/kbench.py --kernel $1 --stage $2 --iters 20 2>&1 | grep "per call" || exit 1; done
