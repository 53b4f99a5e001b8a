#!/usr/bin/env bash
# Fused FPN top: front-end parity, then the default bench with the fused launch and with the two-layer path.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontend.py -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_fe.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_fe.log; grep -E "FAILED|Error" gpurun_out/pytest_fe.log | head -5
[ $rc -eq 0 ] || exit $rc
for v in 1 0 1; do
  DAMVS_FPN_TOP_FUSED=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_fpn.log 2>&1 || { tail -5 gpurun_out/bench_fpn.log; exit 1; }
  echo "fused=$v: $(grep '^{"metric"' gpurun_out/bench_fpn.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["ms_per_stage"]["features"])')"
done
