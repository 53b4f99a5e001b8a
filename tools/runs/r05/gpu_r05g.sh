#!/bin/bash
# Round-5 g: per-layer CostRegNet times at cfgC B=4, fp32 and bf16 (tools/unet_layers.py).
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/unet_layers.py --dtype f32 > gpurun_out/unet_layers_f32.txt 2>&1 || exit $?
timeout -k 10 240 python -u tools/unet_layers.py --dtype bf16 > gpurun_out/unet_layers_bf16.txt 2>&1 || exit $?
grep total gpurun_out/unet_layers_*.txt
