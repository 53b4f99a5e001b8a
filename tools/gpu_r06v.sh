#!/bin/bash
# Round-6: conv0 on the depth-split kernel with input planes 2 / 3 / 4 ahead (-DDAMVS_DZ_AHEAD), every CIN
# (DAMVS_CONV0_DZ=1), against the default kernels.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06v}
timeout -k 10 300 python -u tools/unet_layers.py --dtype f32 --only conv0 > gpurun_out/r06/${T}_default.txt 2>&1 || exit 3
echo "default"; grep conv0 gpurun_out/r06/${T}_default.txt
for v in 2 3 4; do
  if [ $v = 2 ]; then L=""; else L=$R/damvsnet_amd/ab/libdamvs_dz$v.so; fi
  DAMVS_LIB=$L DAMVS_CONV0_DZ=1 timeout -k 10 300 python -u tools/unet_layers.py --dtype f32 --only conv0 > gpurun_out/r06/${T}_dz_ahead$v.txt 2>&1 || exit 3
  echo "dz ahead $v"; grep conv0 gpurun_out/r06/${T}_dz_ahead$v.txt
done
for v in "2,1" "4,2" "2,2"; do
  DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_dz3.so DAMVS_CONV0_DZ=$v timeout -k 10 300 python -u tools/unet_layers.py --dtype f32 --only conv0 --stages 2,3 > gpurun_out/r06/${T}_dz3_$v.txt 2>&1 || exit 3
  echo "dz ahead 3 shape $v"; grep conv0 gpurun_out/r06/${T}_dz3_$v.txt
done
