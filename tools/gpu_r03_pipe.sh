#!/usr/bin/env bash
# U-Net kernel changes: conv3d gather kernel with one-chunk-ahead loads (DAMVS_CONV3D_PIPE=0 restores it) and conv0
# walking input planes (DAMVS_CONV0_REUSE=0 restores the output-plane walk): U-Net parity suites (incl. the bitwise
# kernel-vs-kernel test), then bench A/B (in-pipeline U-Net ms per stage), two rounds
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_streams.py > gpurun_out/pytest_pipe.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_pipe.log; [ $rc -eq 0 ] || exit $rc
for v in X=1 DAMVS_CONV3D_KG1=0 X=1 DAMVS_CONV3D_KG1=0; do
  env $v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { echo "bench $v failed"; tail -3 gpurun_out/bench_ab.err; exit 1; }
  python - "$v" gpurun_out/bench_ab.json <<'PY' | tee -a gpurun_out/ab_unet.jsonl
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
hp = d["hot_path_roofline"]["per_stage"]
print(json.dumps({"env": sys.argv[1], "maps_s": d["value"], "unet_ms": [hp[s]["kernels"]["unet"]["ms"] for s in ("stage1", "stage2", "stage3")],
                  "warp_ms": [hp[s]["kernels"]["warp"]["ms"] for s in ("stage1", "stage2", "stage3")]}), flush=True)
PY
done
