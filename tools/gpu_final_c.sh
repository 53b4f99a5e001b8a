#!/bin/bash
# Round-6 checkpoint C: in-pipeline PMC of the stage-2 warp (the roofline kernel), bf16 and fp32 (tools/pmc_warp_inpipe.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06/pmc
timeout -k 10 900 python -u tools/pmc_warp_inpipe.py --out gpurun_out/r06/pmc/inpipe_bf16 > gpurun_out/r06/pmc/inpipe_bf16.log 2>&1 || { tail -5 gpurun_out/r06/pmc/inpipe_bf16.log; exit 3; }
PMC_DTYPE=f32 timeout -k 10 900 python -u tools/pmc_warp_inpipe.py --out gpurun_out/r06/pmc/inpipe_f32 > gpurun_out/r06/pmc/inpipe_f32.log 2>&1 || { tail -5 gpurun_out/r06/pmc/inpipe_f32.log; exit 4; }
tail -12 gpurun_out/r06/pmc/inpipe_bf16.log; tail -12 gpurun_out/r06/pmc/inpipe_f32.log
