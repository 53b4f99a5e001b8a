#!/usr/bin/env bash
# session re-entry check: full GPU suite with the measured errors printed (-s), then the default bench
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/pytest_gpu_o.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_o.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench_o.json 2> gpurun_out/bench_o.err || { tail -3 gpurun_out/bench_o.err; exit 1; }
tail -1 gpurun_out/bench_o.json | cut -c1-300
