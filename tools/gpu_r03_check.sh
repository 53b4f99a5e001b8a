#!/usr/bin/env bash
# final-code check: the whole GPU suite, smoke() and the default bench line
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/pytest_gpu_final.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { tail -5 gpurun_out/smoke_final.log; exit 1; }
tail -2 gpurun_out/smoke_final.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -3 gpurun_out/bench_final.err; exit 1; }
tail -1 gpurun_out/bench_final.json | cut -c1-250
