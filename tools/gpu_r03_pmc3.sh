#!/usr/bin/env bash
# PMC counters of the stage-3 and stage-1 warps in the pipeline (one-lane / channel-split defaults and the corner-pair
# kernel): clock, TA busy, L1 tag lookups, L2 hit, VALU instructions
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
run() {  # name kernel grid [env]
  local name=$1 kern=$2 grid=$3; shift 3
  env "$@" PMC_WARP_KERNEL="$kern" PMC_WARP_GRID="$grid" timeout -k 10 500 python -u tools/pmc_warp_inpipe.py --out /tmp/pmc_$name --passes 0,1,2,3 > gpurun_out/pmc_$name.log 2>&1 || { tail -5 gpurun_out/pmc_$name.log; return 1; }
  cp /tmp/pmc_$name/pmc_warp_inpipe.json gpurun_out/pmc_$name.json
  python - gpurun_out/pmc_$name.json "$name" <<'PY'
import json, sys
s = json.load(open(sys.argv[1]))["summary"]["pipeline"]
print(sys.argv[2], {k: round(v, 3) for k, v in s.items() if k in ("ms", "effective_clock_GHz", "TA_busy_frac",
      "TA_cycles_per_buffer_read_instr", "l1_tag_lookups_per_read_instr", "l2_hit_rate")},
      "VALU/voxel-wave %.1f" % (s.get("SQ_INSTS_VALU", 0) / max(1, s.get("SQ_WAVES", 1))))
PY
}
run s3_onelane "warp_aggregate_kernel<unsigned short, 8," 7577600 X=0 && \
run s3_pair "warp_pair_kernel<unsigned short, 8," 15155200 DAMVS_WARP_PAIR=1 && \
run s1_split "warp_split_kernel<unsigned short, 32," 1894400 X=0
