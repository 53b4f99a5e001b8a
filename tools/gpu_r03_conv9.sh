#!/usr/bin/env bash
# conv9 variants: U-Net parity (incl. the bitwise kernel-vs-kernel test), then bench A/B of the in-pipeline U-Net
# time: A fragments in LDS for two waves per SIMD (DAMVS_DECONV_A_LDS=1) against registers, three rounds
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/pytest_conv9.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_conv9.log; [ $rc -eq 0 ] || exit $rc
for v in X=1 DAMVS_DECONV_A_LDS=1 X=1 DAMVS_DECONV_A_LDS=1 X=1 DAMVS_DECONV_A_LDS=1; do
  env $v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { echo "bench $v failed"; tail -3 gpurun_out/bench_ab.err; exit 1; }
  python - "$v" gpurun_out/bench_ab.json <<'PY' | tee -a gpurun_out/ab_conv9.jsonl
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
hp = d["hot_path_roofline"]["per_stage"]
print(json.dumps({"env": sys.argv[1], "maps_s": d["value"], "unet_ms": [hp[s]["kernels"]["unet"]["ms"] for s in ("stage1", "stage2", "stage3")]}), flush=True)
PY
done
