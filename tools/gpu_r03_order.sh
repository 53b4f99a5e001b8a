#!/usr/bin/env bash
# Warp block-order A/B (DAMVS_WARP_ORDER 0 / 1 / 2), default bench config, alternating: in-pipeline stage-1/2/3 warp ms.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
for rep in 1 2; do
  for o in 0 1 2; do
    DAMVS_WARP_ORDER=$o timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_order${o}_$rep.json 2> gpurun_out/bench_order${o}_$rep.err || { echo "order $o failed"; tail -3 gpurun_out/bench_order${o}_$rep.err; exit 1; }
    python - "$o" "gpurun_out/bench_order${o}_$rep.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
hp = d["hot_path_roofline"]["per_stage"]
print("order", sys.argv[1], "maps/s", d["value"], "warp ms", [hp[s]["kernels"]["warp"]["ms"] for s in ("stage1", "stage2", "stage3")], flush=True)
PY
  done
done
