#!/bin/bash
# Round-6: the stride-2 5x5 LDS conv2d kernel (FeatureNet conv1.0 / conv2.0): front-end GPU tests, kbench2d FA / FB
# against DAMVS_CONV2D_LDS_S2=0 (the 32-K / 16-K gather kernel), then bench A/B lines of both dtypes.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06o}
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_frontend.py > gpurun_out/r06/${T}_pytest_frontend.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r06/${T}_pytest_frontend.log; [ $rc -eq 0 ] || exit $rc
for dt in f32 bf16; do
  for v in 1 0; do
    DAMVS_CONV2D_LDS_S2=$v timeout -k 10 200 python -u tools/kbench2d.py --dtype $dt --only FA,FB,I > gpurun_out/r06/${T}_k2d_${dt}_s2$v.txt 2>&1 || exit 7
    echo "$dt LDS_S2=$v"; grep -E "^(FA|FB|I) " gpurun_out/r06/${T}_k2d_${dt}_s2$v.txt
  done
done
TAG=${T} bash tools/gpu_ab.sh "s2 f32|DAMVS_X=1|--dtype f32" "gather f32|DAMVS_CONV2D_LDS_S2=0|--dtype f32" "s2 bf16|DAMVS_X=1|--no-parity-path" "gather bf16|DAMVS_CONV2D_LDS_S2=0|--no-parity-path"
