#!/bin/bash
# Round-6: fp32 stride-2 GeoBlock convs on the wide kernel (default) against the 32-K gather kernel
# (DAMVS_CONV2D_WIDE_S2=0): kbench2d E / H and the fp32 bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06w}
for v in 1 0; do
  DAMVS_CONV2D_WIDE_S2=$v timeout -k 10 200 python -u tools/kbench2d.py --dtype f32 --only E,H > gpurun_out/r06/${T}_k2d_f32_s2$v.txt 2>&1 || exit 7
  echo "WIDE_S2=$v"; grep -E "^(E|H) " gpurun_out/r06/${T}_k2d_f32_s2$v.txt
done
TAG=${T} bash tools/gpu_ab.sh "f32 wide|DAMVS_X=1|--dtype f32" "f32 gather|DAMVS_CONV2D_WIDE_S2=0|--dtype f32"
