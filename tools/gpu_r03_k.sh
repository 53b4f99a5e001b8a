#!/usr/bin/env bash
# split warp at stage 1 (NHWC, 4 lanes per voxel) vs the blocked one-lane form: parity subset + A/B bench
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_streams.py > gpurun_out/pytest_split1.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_split1.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for sp in 1 0; do
    DAMVS_WARP_SPLIT=$sp timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_s1split${sp}_$rep.json 2> gpurun_out/bench_s1split${sp}_$rep.err || { echo "bench split=$sp failed"; tail -3 gpurun_out/bench_s1split${sp}_$rep.err; exit 1; }
    python - "$sp" "gpurun_out/bench_s1split${sp}_$rep.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
hp = d["hot_path_roofline"]["per_stage"]
print("split", sys.argv[1], "maps/s", d["value"], "warp ms", [hp[s]["kernels"]["warp"]["ms"] for s in ("stage1", "stage2", "stage3")], "per-map hot", d["hot_path_roofline"]["per_map"], flush=True)
PY
  done
done
