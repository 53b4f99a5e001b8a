#!/usr/bin/env bash
# conv2d_wide LDS epilogue + transposed-s1 tap order: front-end parity, then bench A/B (DAMVS_CONV2D_WIDE=0 as
# the reference point is not the old epilogue; the layer table shows the per-layer change)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_frontend.py tests/test_gpu_parity.py -k "not fullres" > gpurun_out/pytest_fe.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_fe.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_epi_$rep.json 2> gpurun_out/bench_epi_$rep.err || { tail -3 gpurun_out/bench_epi_$rep.err; exit 1; }
  python - "gpurun_out/bench_epi_$rep.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("maps/s", d["value"], "ms/stage", d["ms_per_stage"], flush=True)
PY
done
timeout -k 10 200 python tools/layer_times.py --top 40 > gpurun_out/layer_times_epi.txt 2>&1 && head -2 gpurun_out/layer_times_epi.txt | tail -1
