#!/bin/bash
# Round-6: fp32 conv0 per stage (tools/unet_layers.py) and its PMC passes.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06u}
timeout -k 10 300 python -u tools/unet_layers.py --dtype f32 --only conv0 > gpurun_out/r06/${T}_layers_conv0_f32.txt 2>&1 || exit 3
grep conv0 gpurun_out/r06/${T}_layers_conv0_f32.txt
bash tools/pmc_cmd.sh r06/${T}_pmc_conv0_f32 tools/unet_layers.py --dtype f32 --only conv0 --iters 3 > /dev/null && cat gpurun_out/r06/${T}_pmc_conv0_f32/table.txt
