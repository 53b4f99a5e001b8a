#!/usr/bin/env bash
# Occupancy-cap A/B: front-end / U-Net / warp parity subset on the capped build, then the default bench alternating
# the capped build with the uncapped one (damvsnet_amd/ab/libdamvs_noocc.so, tools/build_variant.sh noocc -DDAMVS_NO_OCC).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_frontend.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > gpurun_out/pytest_occ.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_occ.log | tail -8
[ $rc -eq 0 ] || exit $rc
for v in cap noocc cap noocc; do
  if [ $v = cap ]; then unset DAMVS_LIB; else export DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_noocc.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/bench_occ.log 2>&1 || { tail -5 gpurun_out/bench_occ.log; exit 1; }
  echo "$v: $(grep '^{"metric"' gpurun_out/bench_occ.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); h=d["hot_path_roofline"]["per_stage"]; print(d["value"], d["ms_per_step"], {k: round(v, 3) for k, v in d["ms_per_stage"].items() if v > 0.5}, [[round(h[s]["kernels"][k]["ms"], 3) for k in ("warp", "unet")] for s in h])')"
done
