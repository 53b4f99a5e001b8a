#!/usr/bin/env bash
# Stage-1 (32-channel) warp on the runtime view pipeline: warp parity subset, then cfgC / cfgD benches alternating the
# tree with DAMVS_WARP_PIPE32=0 (the generic view loop).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_p32.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_p32.log | tail -8
[ $rc -eq 0 ] || exit $rc
line() { python -c 'import json,sys; d=json.loads(sys.stdin.read()); h=d["hot_path_roofline"]["per_stage"]; print(d["value"], d["ms_per_step"], [round(h[s]["kernels"]["warp"]["ms"], 3) for s in h])'; }
for c in cfgC cfgD; do
  for v in 1 0 1 0; do
    DAMVS_WARP_PIPE32=$v timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --steps 20 > gpurun_out/bench_p.log 2>&1 || { tail -5 gpurun_out/bench_p.log; exit 1; }
    echo "$c pipe32=$v: $(grep '^{"metric"' gpurun_out/bench_p.log | tail -1 | line)"
  done
done
