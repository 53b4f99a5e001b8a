#!/bin/bash
# Round-6: thin stride-1 3x3 layers on the LDS kernel (default) against the halo / gather kernels (DAMVS_CONV2D_NO_LDS=1).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06ab}
for dt in f32 bf16; do
  for v in 0 1; do
    DAMVS_CONV2D_NO_LDS=$v timeout -k 10 200 python -u tools/kbench2d.py --dtype $dt --only A,U,C,FC,FD,V > gpurun_out/r06/${T}_k2d_${dt}_nolds$v.txt 2>&1 || exit 7
  done
  echo "== $dt"; paste gpurun_out/r06/${T}_k2d_${dt}_nolds0.txt gpurun_out/r06/${T}_k2d_${dt}_nolds1.txt | grep " us" | awk -F'\t' '{print $1 " || " $2}' | cut -c1-140
done
