#!/usr/bin/env bash
# Checkpoint: full GPU suite, default bench line, kernel-trace profile of the bench (per-step table).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_cfgC.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench_cfgC.log | cut -c1-600; echo
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh
