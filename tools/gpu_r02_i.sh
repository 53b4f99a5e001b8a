#!/usr/bin/env bash
# Checkpoint: full GPU suite, default bench line (with the CPU baseline), cfgD / cfgE bench lines, kernel-trace
# profiles of the default bench (tools/gpu_prof.sh).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_cfgC.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench_cfgC.log | cut -c1-300; echo
[ $rc -eq 0 ] || exit $rc
for c in cfgD cfgE; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1 || { tail -5 gpurun_out/bench_$c.log; exit 1; }
  grep '^{"metric"' gpurun_out/bench_$c.log | tail -1 > gpurun_out/bench_${c}_line.json
  echo "$c: $(cut -c1-200 gpurun_out/bench_${c}_line.json)"
done
bash tools/gpu_prof.sh
