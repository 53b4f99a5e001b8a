#!/usr/bin/env bash
# Round-2 first GPU pass: GPU tests, cfgC bench (no CPU leg), cfgD / cfgE bench lines, kernel trace.
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -20
[ $rc -eq 0 ] || exit $rc
for c in cfgC cfgD cfgE; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1; rc=$?
  echo "bench $c rc=$rc"; tail -c 600 gpurun_out/bench_$c.log; echo
  [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_cfgC" -o run -- \
  python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/prof_cfgC.log" 2>&1; rc=$?
echo "prof rc=$rc"
exit $rc
