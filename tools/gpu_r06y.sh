#!/bin/bash
# Round-6: one-row stride-2 tiles by default, fp32 64-channel stride-2 layers on the gather kernel: front-end tests,
# kbench2d E / H, fp32 bench lines against the 2-row tiles (DAMVS_WIDE_S2R1=0).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06y}
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_frontend.py > gpurun_out/r06/${T}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r06/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/kbench2d.py --dtype f32 --only E,H,K > gpurun_out/r06/${T}_k2d_f32.txt 2>&1 || exit 7
grep -E "^(E|H|K) " gpurun_out/r06/${T}_k2d_f32.txt
TAG=${T} bash tools/gpu_ab.sh "f32|DAMVS_X=1|--dtype f32" "f32 2row|DAMVS_WIDE_S2R1=0|--dtype f32" "f32 b|DAMVS_X=1|--dtype f32"
