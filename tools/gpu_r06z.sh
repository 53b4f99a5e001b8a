#!/bin/bash
# Round-6: fp32 stride-1 64-channel wide block against the 32-K gather kernel (DAMVS_CONV2D_WIDE64=0): kbench2d K / L / R,
# fp32 bench lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06z}
for v in 1 0; do
  DAMVS_CONV2D_WIDE64=$v timeout -k 10 200 python -u tools/kbench2d.py --dtype f32 --only K,L,R > gpurun_out/r06/${T}_k2d_f32_w64$v.txt 2>&1 || exit 7
  echo "WIDE64=$v"; grep -E "^(K|L|R) " gpurun_out/r06/${T}_k2d_f32_w64$v.txt
done
TAG=${T} bash tools/gpu_ab.sh "f32|DAMVS_X=1|--dtype f32" "f32 w64off|DAMVS_CONV2D_WIDE64=0|--dtype f32" "f32 b|DAMVS_X=1|--dtype f32" "f32 w64off b|DAMVS_CONV2D_WIDE64=0|--dtype f32"
