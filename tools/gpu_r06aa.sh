#!/bin/bash
# Round-6: fp32 narrow layers on the halo kernels (default) against the 32-K gather kernel (DAMVS_CONV2D_HALO32=0):
# kbench2d and fp32 bench lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06aa}
for v in 1 0; do
  DAMVS_CONV2D_HALO32=$v timeout -k 10 200 python -u tools/kbench2d.py --dtype f32 --only C,G,M,O,P,Q,G4,M4,J,T > gpurun_out/r06/${T}_k2d_f32_h$v.txt 2>&1 || exit 7
done
paste gpurun_out/r06/${T}_k2d_f32_h1.txt gpurun_out/r06/${T}_k2d_f32_h0.txt | grep " us" | awk -F'\t' '{print $1 " || " $2}' | cut -c1-140
TAG=${T} bash tools/gpu_ab.sh "f32|DAMVS_X=1|--dtype f32" "f32 h0|DAMVS_CONV2D_HALO32=0|--dtype f32" "f32 b|DAMVS_X=1|--dtype f32" "f32 h0 b|DAMVS_CONV2D_HALO32=0|--dtype f32"
