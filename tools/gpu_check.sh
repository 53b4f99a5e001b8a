#!/usr/bin/env bash
# One GPU-box call: parity tests, bench lines and a kernel-trace profile, each step under its own time limit, the
# chain stopping at the first failure. Outputs under gpurun_out/<TAG>_*.
#   TAG=r04a TESTS="tests/test_gpu_parity.py -k fp32" BENCH="bf16 f32" PROF=f32 tools/gpu_check.sh
# TESTS: pytest selection ("" skips; "all" = tests -m gpu); BENCH: dtypes for a 20-step bench line each; PROF: dtype
# for a rocprofv3 --kernel-trace --stats pass over a 5-step bench (one stream); EXTRA: bench arguments for all lines.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
TAG="${TAG:-run}"
TESTS="${TESTS-}"
BENCH="${BENCH-}"
PROF="${PROF-}"
EXTRA="${EXTRA-}"
if [ -n "$TESTS" ]; then
  [ "$TESTS" = "all" ] && TESTS="tests -m gpu"
  timeout -k 10 1000 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread $TESTS \
    > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"
  grep -E "FAILED|ERROR|passed|failed|e2e |bf16 mean|fp32 max|split " gpurun_out/${TAG}_pytest.log | tail -40
  [ $rc -eq 0 ] || exit $rc
fi
for dt in $BENCH; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --dtype $dt --no-cpu-baseline $EXTRA \
    > gpurun_out/${TAG}_bench_$dt.json 2> gpurun_out/${TAG}_bench_$dt.err; rc=$?
  echo "bench $dt rc=$rc"; tail -c 600 gpurun_out/${TAG}_bench_$dt.json; echo
  [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_bench_$dt.err; exit $rc; }
done
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_prof" -o run -- \
    python "$R/bench.py" --steps 5 --warmup 2 --streams 1 --dtype $PROF --no-cpu-baseline --no-shard-latency $EXTRA \
    > "$R/gpurun_out/${TAG}_prof_bench.log" 2>&1; rc=$?
  echo "prof rc=$rc"
  [ $rc -eq 0 ] || { tail -20 "$R/gpurun_out/${TAG}_prof_bench.log"; exit $rc; }
  cd "$R"
  f=$(find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" | head -1)
  [ -n "$f" ] && python tools/prof_steps.py "$f" 2 5 > gpurun_out/${TAG}_prof_steps.txt && head -45 gpurun_out/${TAG}_prof_steps.txt
fi
exit 0
