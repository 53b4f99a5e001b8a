#!/usr/bin/env bash
# (1) warp pixel-block shape A/B (DAMVS_WARP_TILE="rows,strip width") and (2) stride-2 wide conv2d A/B
# (DAMVS_CONV2D_WIDE_S2=0 restores the gather kernel): parity suites first, then the bench's in-pipeline times
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_frontend.py > gpurun_out/pytest_fe_s2.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_fe_s2.log; [ $rc -eq 0 ] || exit $rc
DAMVS_WARP_TILE=4,256 timeout -k 10 400 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_sharded.py > gpurun_out/pytest_tile.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_tile.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config cfgD --shard gather --emulate 4 --steps 2 --warmup 1 > gpurun_out/bench_shard_gather.json 2> gpurun_out/bench_shard_gather.err || { tail -3 gpurun_out/bench_shard_gather.err; exit 1; }
tail -1 gpurun_out/bench_shard_gather.json | cut -c1-600
for v in "" "DAMVS_CONV2D_WIDE_S2=0" "DAMVS_CONV2D_WIDE64=0" "DAMVS_WARP_TILE=2,0" "DAMVS_WARP_TILE=4,0" "DAMVS_WARP_TILE=4,256" "DAMVS_WARP_TILE=4,128" "DAMVS_WARP_TILE=2,256" "DAMVS_WARP_TILE=4,512" "" "DAMVS_CONV2D_WIDE_S2=0" "DAMVS_CONV2D_WIDE64=0"; do
  env $v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { echo "bench $v failed"; tail -3 gpurun_out/bench_ab.err; exit 1; }
  python - "$v" gpurun_out/bench_ab.json <<'PY' | tee -a gpurun_out/ab_tile_s2.jsonl
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
hp = d["hot_path_roofline"]["per_stage"]
m = d["ms_per_stage"]
print(json.dumps({"env": sys.argv[1], "maps_s": d["value"], "warp_ms": [hp[s]["kernels"]["warp"]["ms"] for s in ("stage1", "stage2", "stage3")],
                  "geofusion_ms": [m["stage2.geofusion"], m["stage3.geofusion"]]}), flush=True)
PY
done
