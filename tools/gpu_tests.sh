#!/usr/bin/env bash
# GPU tests only: tools/gpu_tests.sh [pytest args...]  (default: the whole -m gpu suite)
# One pytest process, its own time limit, per-test timeout; output in gpurun_out/pytest_gpu.log.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
args=("$@")
[ ${#args[@]} -eq 0 ] && args=(tests -m gpu)
timeout -k 10 1000 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
  "${args[@]}" > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"
grep -E "PASSED|FAILED|ERROR|passed|failed|e2e |bf16 mean|fp32 max" gpurun_out/pytest_gpu.log | tail -60
exit $rc
