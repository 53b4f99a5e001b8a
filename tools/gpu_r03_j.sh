#!/usr/bin/env bash
# in-pipeline PMC of the split vs one-lane stage-2 warps (raw rocprof output under /tmp; JSON summaries to gpurun_out)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u tools/pmc_warp_inpipe.py --out /tmp/pmc_inpipe_split > gpurun_out/pmc_inpipe_split.log 2>&1; echo "split rc=$?"; cp /tmp/pmc_inpipe_split/pmc_warp_inpipe.json gpurun_out/pmc_warp_inpipe_split.json &&
DAMVS_WARP_SPLIT=0 timeout -k 10 900 python -u tools/pmc_warp_inpipe.py --out /tmp/pmc_inpipe_onelane > gpurun_out/pmc_inpipe_onelane.log 2>&1; echo "onelane rc=$?"; cp /tmp/pmc_inpipe_onelane/pmc_warp_inpipe.json gpurun_out/pmc_warp_inpipe_onelane.json
tail -3 gpurun_out/pmc_inpipe_split.log gpurun_out/pmc_inpipe_onelane.log
