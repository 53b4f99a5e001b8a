#!/bin/bash
# Round-6: sub-batch stream offsets (sub-batch 2 starts when sub-batch 1 reaches a stage-hook point): the stream
# bitwise tests, then bench A/B lines of both dtypes.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06s}
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_streams.py -k sub_batches > gpurun_out/r06/${T}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r06/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=${T} bash tools/gpu_ab.sh "f32 none|DAMVS_X=1|--dtype f32" "f32 s1hyp|DAMVS_X=1|--dtype f32 --stream-offset stage1.hypotheses" "f32 s1dn|DAMVS_X=1|--dtype f32 --stream-offset stage1.depthnet" "f32 s2geo|DAMVS_X=1|--dtype f32 --stream-offset stage2.geofusion" "f32 none2|DAMVS_X=1|--dtype f32" "f32 s1hyp2|DAMVS_X=1|--dtype f32 --stream-offset stage1.hypotheses" "bf16 none|DAMVS_X=1|--no-parity-path" "bf16 s1hyp|DAMVS_X=1|--no-parity-path --stream-offset stage1.hypotheses"
