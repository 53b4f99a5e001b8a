#!/usr/bin/env bash
# warp pixel-block shape A/B (DAMVS_WARP_TILE="rows,strip width"): warp parity suite with a tiled mapping, then the
# bench's in-pipeline warp times per stage for each shape (default first and last)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
DAMVS_WARP_TILE=4,256 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "warp or depthnet or forward" > gpurun_out/pytest_tile.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_tile.log; [ $rc -eq 0 ] || exit $rc
for t in 0 2,0 4,0 4,256 4,128 2,256 4,512 0; do
  DAMVS_WARP_TILE=$t timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_tile.json 2> gpurun_out/bench_tile.err || { echo "bench tile=$t failed"; tail -3 gpurun_out/bench_tile.err; exit 1; }
  python - "$t" gpurun_out/bench_tile.json <<'PY' | tee -a gpurun_out/tile_ab.jsonl
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
hp = d["hot_path_roofline"]["per_stage"]
print(json.dumps({"tile": sys.argv[1], "maps_s": d["value"], "warp_ms": [hp[s]["kernels"]["warp"]["ms"] for s in ("stage1", "stage2", "stage3")]}), flush=True)
PY
done
