#!/usr/bin/env bash
# full GPU suite with the 16-row warp tiles as the default, then tile-row A/B (two rounds)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/pytest_gpu_tile16.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu_tile16.log; [ $rc -eq 0 ] || exit $rc
for v in 16,0 32,0 64,0 8,0 16,0 32,0 64,0 8,0; do
  DAMVS_WARP_TILE=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { echo "bench $v failed"; tail -3 gpurun_out/bench_ab.err; exit 1; }
  python - "$v" gpurun_out/bench_ab.json <<'PY' | tee -a gpurun_out/ab_tile3.jsonl
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
hp = d["hot_path_roofline"]["per_stage"]
print(json.dumps({"tile": sys.argv[1], "maps_s": d["value"], "warp_ms": [hp[s]["kernels"]["warp"]["ms"] for s in ("stage1", "stage2", "stage3")]}), flush=True)
PY
done
