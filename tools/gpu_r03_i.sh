#!/usr/bin/env bash
# split warp occupancy A/B (LDS pad caps blocks per CU), then in-pipeline PMC of split vs one-lane warps
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
for pad in 0 40000 65536 0 40000 65536; do
  DAMVS_WARP_LDS_PAD=$pad timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_pad$pad.json 2> gpurun_out/bench_pad$pad.err || { echo "bench pad=$pad failed"; tail -3 gpurun_out/bench_pad$pad.err; exit 1; }
  python - "$pad" "gpurun_out/bench_pad$pad.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
hp = d["hot_path_roofline"]["per_stage"]
print("pad", sys.argv[1], "maps/s", d["value"], "warp ms", [hp[s]["kernels"]["warp"]["ms"] for s in ("stage1", "stage2", "stage3")], flush=True)
PY
done
timeout -k 10 900 python -u tools/pmc_warp_inpipe.py --out gpurun_out/pmc_inpipe_split > gpurun_out/pmc_inpipe_split.log 2>&1 && echo "pmc split done" &&
DAMVS_WARP_SPLIT=0 timeout -k 10 900 python -u tools/pmc_warp_inpipe.py --out gpurun_out/pmc_inpipe_onelane > gpurun_out/pmc_inpipe_onelane.log 2>&1 && echo "pmc one-lane done"
