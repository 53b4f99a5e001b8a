#!/bin/bash
# Round-6: prob_regress staging by plane-invariant buffer-load offsets: regression / prob parity tests, the isolated
# fp32 prob bench, the fp32 bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06r}
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "regress or prob or stage_isolated or depthnet" > gpurun_out/r06/${T}_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r06/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/kbench_prob.py 20 f32 > gpurun_out/r06/${T}_kbench_prob_f32.jsonl 2>&1 || exit 3
grep valu gpurun_out/r06/${T}_kbench_prob_f32.jsonl
TAG=${T} bash tools/gpu_ab.sh "f32|DAMVS_X=1|--dtype f32" "f32b|DAMVS_X=1|--dtype f32"
