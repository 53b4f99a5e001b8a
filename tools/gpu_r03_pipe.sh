#!/usr/bin/env bash
# conv3d gather kernel with one-chunk-ahead loads: U-Net parity suites, then per-layer U-Net times and bench A/B
# (DAMVS_CONV3D_PIPE=0 restores the unpipelined kernel)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_streams.py > gpurun_out/pytest_pipe.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_pipe.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  DAMVS_CONV3D_PIPE=$v timeout -k 10 300 bash tools/gpu_unet_layers.sh > gpurun_out/unet_layers_pipe$v.txt 2>&1 || { echo "unet layers $v failed"; tail -5 gpurun_out/unet_layers_pipe$v.txt; exit 1; }
done
for v in 1 0 1 0; do
  DAMVS_CONV3D_PIPE=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { echo "bench $v failed"; tail -3 gpurun_out/bench_ab.err; exit 1; }
  python - "$v" gpurun_out/bench_ab.json <<'PY' | tee -a gpurun_out/ab_pipe.jsonl
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
hp = d["hot_path_roofline"]["per_stage"]
print(json.dumps({"conv3d_pipe": sys.argv[1], "maps_s": d["value"], "unet_ms": [hp[s]["kernels"]["unet"]["ms"] for s in ("stage1", "stage2", "stage3")]}), flush=True)
PY
done
