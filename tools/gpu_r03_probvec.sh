#!/usr/bin/env bash
# 16-byte prob-volume stores and the stride-2 64-channel wide conv: parity + front-end suites, bench A/B
# (DAMVS_PROB_VEC=0: 4-byte stores; DAMVS_CONV2D_WIDE64=0: the 64-channel layers on the gather kernel), then the env sweep
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_frontend.py > gpurun_out/pytest_probvec.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_probvec.log; [ $rc -eq 0 ] || exit $rc
for v in X=1 DAMVS_PROB_VEC=0 DAMVS_CONV2D_WIDE64=0 X=1 DAMVS_PROB_VEC=0 DAMVS_CONV2D_WIDE64=0; do
  env $v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { echo "bench $v failed"; tail -3 gpurun_out/bench_ab.err; exit 1; }
  python - "$v" gpurun_out/bench_ab.json <<'PY' | tee -a gpurun_out/ab_probvec.jsonl
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
hp = d["hot_path_roofline"]["per_stage"]
m = d["ms_per_stage"]
print(json.dumps({"env": sys.argv[1], "maps_s": d["value"], "regress_ms": [hp[s]["kernels"]["regress"]["ms"] for s in ("stage1", "stage2", "stage3")],
                  "geofusion": [m["stage2.geofusion"], m["stage3.geofusion"]]}), flush=True)
PY
done
bash tools/gpu_r03_sweep.sh > gpurun_out/sweep_r03.txt 2>&1; tail -34 gpurun_out/sweep_r03.txt
