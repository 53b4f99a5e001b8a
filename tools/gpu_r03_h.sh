#!/usr/bin/env bash
# split warp: parity subset, then A/B bench (split on / off)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "warp or homo or depthnet or forward" > gpurun_out/pytest_split.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_split.log; grep "warp split\|homo_warping C" gpurun_out/pytest_split.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for sp in 1 0; do
    DAMVS_WARP_SPLIT=$sp timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_split${sp}_$rep.json 2> gpurun_out/bench_split${sp}_$rep.err || { echo "bench split=$sp failed"; tail -3 gpurun_out/bench_split${sp}_$rep.err; exit 1; }
    python - "$sp" "gpurun_out/bench_split${sp}_$rep.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
hp = d["hot_path_roofline"]["per_stage"]
print("split", sys.argv[1], "maps/s", d["value"], "warp ms", [hp[s]["kernels"]["warp"]["ms"] for s in ("stage1", "stage2", "stage3")], "frac", d["roofline"]["frac"], flush=True)
PY
  done
done
