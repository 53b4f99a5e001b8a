#!/usr/bin/env bash
# 4-column plane-only conv kernel: front-end suite (incl. the bitwise test against the one-column kernel), then bench
# A/B of the front-end phases (DAMVS_PLANES4=0 restores the one-column kernel), two rounds
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_frontend.py > gpurun_out/pytest_planes4.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_planes4.log; [ $rc -eq 0 ] || exit $rc
for v in X=1 DAMVS_PLANES4=0 X=1 DAMVS_PLANES4=0; do
  env $v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { echo "bench $v failed"; tail -3 gpurun_out/bench_ab.err; exit 1; }
  python - "$v" gpurun_out/bench_ab.json <<'PY' | tee -a gpurun_out/ab_planes4.jsonl
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
m = d["ms_per_stage"]
print(json.dumps({"env": sys.argv[1], "maps_s": d["value"], "features": m["features"], "geofusion": [m["stage2.geofusion"], m["stage3.geofusion"]]}), flush=True)
PY
done
