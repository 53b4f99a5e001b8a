#!/bin/bash
# Round-6: (1) the fp32 rolling wide loop with two q-rows per wave (DAMVS_WIDE_RS2=1) against one; (2) sub-batch stream
# offsets. Front-end and stream tests first, then kbench2d and bench A/B lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06t}
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_frontend.py -k "rolling or layer_vs_torch or geofusion" > gpurun_out/r06/${T}_pytest_frontend.log 2>&1; rc=$?
echo "pytest frontend rc=$rc"; tail -2 gpurun_out/r06/${T}_pytest_frontend.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_streams.py -k sub_batches > gpurun_out/r06/${T}_pytest_streams.log 2>&1; rc=$?
echo "pytest streams rc=$rc"; tail -2 gpurun_out/r06/${T}_pytest_streams.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  DAMVS_WIDE_RS2=$v timeout -k 10 200 python -u tools/kbench2d.py --dtype f32 --only D,F,N,L > gpurun_out/r06/${T}_k2d_f32_rs2$v.txt 2>&1 || exit 7
  echo "RS2=$v"; grep -E "^(D|F|N|L) " gpurun_out/r06/${T}_k2d_f32_rs2$v.txt
done
TAG=${T} bash tools/gpu_ab.sh "f32 rs1|DAMVS_X=1|--dtype f32" "f32 rs2|DAMVS_WIDE_RS2=1|--dtype f32" "f32 s1hyp|DAMVS_X=1|--dtype f32 --stream-offset stage1.hypotheses" "f32 s1dn|DAMVS_X=1|--dtype f32 --stream-offset stage1.depthnet" "f32 rs1b|DAMVS_X=1|--dtype f32" "f32 rs2b|DAMVS_WIDE_RS2=1|--dtype f32" "f32 s1hypb|DAMVS_X=1|--dtype f32 --stream-offset stage1.hypotheses" "bf16 none|DAMVS_X=1|--no-parity-path" "bf16 s1hyp|DAMVS_X=1|--no-parity-path --stream-offset stage1.hypotheses"
