#!/usr/bin/env bash
# stage-2 warp L2 locality: in-pipeline PMC (TA busy, L2 hit, L1->L2 requests) for fewer blocks in flight per CU
# (DAMVS_WARP_LDS_PAD) and shorter depth chunks (DAMVS_WARP_MINBLK), against the default
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
run() {  # name, grid (threads per launch), env...
  local name=$1 grid=$2; shift 2
  env "$@" PMC_WARP_GRID=$grid timeout -k 10 400 python -u tools/pmc_warp_inpipe.py --out gpurun_out/pmc_l2_$name --passes 1,2,3 > gpurun_out/pmc_l2_$name.log 2>&1 || { echo "pmc $name failed"; tail -5 gpurun_out/pmc_l2_$name.log; return 1; }
  echo "== $name"; python -c "import json,sys; d=json.load(open(sys.argv[1]))['summary']['pipeline']; print({k: round(v, 3) if isinstance(v, float) else v for k, v in d.items()})" gpurun_out/pmc_l2_$name/pmc_warp_inpipe.json
}
run default 3788800 DAMVS_WARP_TILE=0 && run tile4 3788800 DAMVS_WARP_TILE=4,0 && run pad54k 3788800 DAMVS_WARP_TILE=0 DAMVS_WARP_LDS_PAD=54000 && run minblk65k 30310400 DAMVS_WARP_TILE=0 DAMVS_WARP_MINBLK=65536
