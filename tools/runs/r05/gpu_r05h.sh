#!/bin/bash
# Round-5 h: the warp gather A/B (tools/gpu_ab_warp_ta.sh), then PMC of conv0 (fp32 and bf16, stages 1-3).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash tools/gpu_ab_warp_ta.sh || exit $?
bash tools/pmc_cmd.sh pmc_conv0_f32 tools/unet_layers.py --dtype f32 --only conv0,conv11 --iters 2 || exit $?
bash tools/pmc_cmd.sh pmc_conv0_bf16 tools/unet_layers.py --dtype bf16 --only conv0,conv11 --iters 2 || exit $?
