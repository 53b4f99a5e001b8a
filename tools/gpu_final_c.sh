#!/bin/bash
# Round-6 checkpoint C: in-pipeline PMC of the stage-2 warp (the roofline kernel), bf16 and fp32 (tools/pmc_warp_inpipe.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06/pmc
timeout -k 10 900 python -u tools/pmc_warp_inpipe.py --out gpurun_out/r06/pmc/inpipe_bf16 > gpurun_out/r06/pmc/inpipe_bf16.log 2>&1 || { tail -5 gpurun_out/r06/pmc/inpipe_bf16.log; exit 3; }
rm -rf gpurun_out/r06/pmc/inpipe_bf16/p[0-9]*  # the rocprofv3 passes (over the 64 MiB copy-back limit); the JSON stays
PMC_DTYPE=f32 timeout -k 10 900 python -u tools/pmc_warp_inpipe.py --out gpurun_out/r06/pmc/inpipe_f32 > gpurun_out/r06/pmc/inpipe_f32.log 2>&1 || { tail -5 gpurun_out/r06/pmc/inpipe_f32.log; exit 4; }
rm -rf gpurun_out/r06/pmc/inpipe_f32/p[0-9]* gpurun_out/prof_default gpurun_out/prof_q
tail -12 gpurun_out/r06/pmc/inpipe_bf16.log; tail -12 gpurun_out/r06/pmc/inpipe_f32.log
