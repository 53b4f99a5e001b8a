#!/usr/bin/env bash
# Stage-2 warp (NHWC 32-byte pixels): unrolled N = 5 view loop vs the runtime one (DAMVS_WARP_RUNTIME_VIEWS=1).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
line() { python -c 'import json,sys; d=json.loads(sys.stdin.read()); h=d["hot_path_roofline"]["per_stage"]; print(d["value"], d["ms_per_step"], [round(h[s]["kernels"]["warp"]["ms"], 3) for s in h])'; }
for v in 0 1 0 1; do
  DAMVS_WARP_RUNTIME_VIEWS=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/bench_rtv.log 2>&1 || { tail -5 gpurun_out/bench_rtv.log; exit 1; }
  echo "runtime_views=$v: $(grep '^{"metric"' gpurun_out/bench_rtv.log | tail -1 | line)"
done
