#!/bin/bash
# Round-6: the fp32 stride-2 128-channel wide block on one-row q-tiles (DAMVS_WIDE_S2R1=1) against the 2-row tiles and
# the 32-K gather kernel (DAMVS_CONV2D_WIDE_S2=0): bitwise test, kbench2d E / H, fp32 bench lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06x}
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_frontend.py -k "one_row or layer_vs_torch" > gpurun_out/r06/${T}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r06/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in "DAMVS_X=1" "DAMVS_WIDE_S2R1=1" "DAMVS_CONV2D_WIDE_S2=0"; do
  env $v timeout -k 10 200 python -u tools/kbench2d.py --dtype f32 --only E,H > gpurun_out/r06/${T}_k2d_${v%%=*}.txt 2>&1 || exit 7
  echo "$v"; grep -E "^(E|H) " gpurun_out/r06/${T}_k2d_${v%%=*}.txt
done
TAG=${T} bash tools/gpu_ab.sh "f32 2row|DAMVS_X=1|--dtype f32" "f32 r1|DAMVS_WIDE_S2R1=1|--dtype f32" "f32 gather|DAMVS_CONV2D_WIDE_S2=0|--dtype f32" "f32 2row b|DAMVS_X=1|--dtype f32" "f32 r1 b|DAMVS_WIDE_S2R1=1|--dtype f32"
