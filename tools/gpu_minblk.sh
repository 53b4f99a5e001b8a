#!/usr/bin/env bash
# In-pipeline warp A/B over the depth-chunk target (DAMVS_WARP_MINBLK: more, shorter depth chunks put fewer image
# rows in flight per XCD), alternating with the default.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
line() { python -c 'import json,sys; d=json.loads(sys.stdin.read()); h=d["hot_path_roofline"]["per_stage"]; print(d["value"], d["ms_per_step"], [round(h[s]["kernels"]["warp"]["ms"], 3) for s in h])'; }
for v in 2048 16384 65536 2048 16384 65536 262144; do
  DAMVS_WARP_MINBLK=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/bench_mb.log 2>&1 || { tail -5 gpurun_out/bench_mb.log; exit 1; }
  echo "minblk=$v: $(grep '^{"metric"' gpurun_out/bench_mb.log | tail -1 | line)"
done
