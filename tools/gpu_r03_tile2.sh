#!/usr/bin/env bash
# warp pixel-block rows A/B, two rounds (DAMVS_WARP_TILE="rows,0": tiles of `rows` rows dealt across the full width;
# 0 = one row-major run of pixels per block)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
for v in 0 4,0 8,0 16,0 0 4,0 8,0 16,0; do
  DAMVS_WARP_TILE=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { echo "bench $v failed"; tail -3 gpurun_out/bench_ab.err; exit 1; }
  python - "$v" gpurun_out/bench_ab.json <<'PY' | tee -a gpurun_out/ab_tile2.jsonl
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
hp = d["hot_path_roofline"]["per_stage"]
print(json.dumps({"tile": sys.argv[1], "maps_s": d["value"], "warp_ms": [hp[s]["kernels"]["warp"]["ms"] for s in ("stage1", "stage2", "stage3")]}), flush=True)
PY
done
bash tools/gpu_r03_l2.sh
