#!/bin/bash
# Whole GPU test suite + short bench (no CPU baseline). Stops at the first fault/timeout.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|Error" gpurun_out/pytest_gpu.log | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/bench_q.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench_q.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['ms_per_stage'], d['roofline']['ms_per_launch'])"
exit $rc
