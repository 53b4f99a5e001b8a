#!/bin/bash
# Round-6: fp32 epilogues with every lane storing its own 16 bytes (conv11, conv9, 2D x-pair layers): parity / stream /
# front-end tests, per-layer times against HEAD (damvsnet_amd/ab/libdamvs_base.so), fp32 bench lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06ac}
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_streams.py tests/test_gpu_frontend.py -k "costreg or unet or conv11 or deconv or stage_isolated or forward or sub_batches or prescale or layer_vs_torch or fpn or featurenet or geofusion" > gpurun_out/r06/${T}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r06/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in new base; do
  if [ $v = new ]; then L=""; else L=$R/damvsnet_amd/ab/libdamvs_base.so; fi
  DAMVS_LIB=$L timeout -k 10 300 python -u tools/unet_layers.py --dtype f32 --only conv11,conv9 > gpurun_out/r06/${T}_unet_$v.txt 2>&1 || exit 3
  echo "$v"; grep -E "conv11|conv9" gpurun_out/r06/${T}_unet_$v.txt
  DAMVS_LIB=$L timeout -k 10 200 python -u tools/kbench2d.py --dtype f32 --only T,Z4,S > gpurun_out/r06/${T}_k2d_$v.txt 2>&1 || exit 4
  grep -E "^(T|Z4|S) " gpurun_out/r06/${T}_k2d_$v.txt
done
TAG=${T} bash tools/gpu_ab.sh "f32 new|DAMVS_X=1|--dtype f32" "f32 base|DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_base.so|--dtype f32" "f32 new b|DAMVS_X=1|--dtype f32" "f32 base b|DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_base.so|--dtype f32"
