#!/bin/bash
# Round-6: front-end GPU tests + kbench2d (idle halo waves; the K32 pipelining A/B build), then the fp32 prob-conv A/B (VALU prob_regress vs
# DAMVS_PROB_MFMA=1) on the fp32 bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06n}
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_frontend.py > gpurun_out/r06/${T}_pytest_frontend.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r06/${T}_pytest_frontend.log; [ $rc -eq 0 ] || exit $rc
for dt in f32 bf16; do
  timeout -k 10 200 python -u tools/kbench2d.py --dtype $dt > gpurun_out/r06/${T}_k2d_$dt.txt 2>&1 || exit 7
  grep -E "^(G|M|O|P|Q|C|G4|M4|FA|FB|I|Z4) " gpurun_out/r06/${T}_k2d_$dt.txt
done
DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_g32pipe.so timeout -k 10 200 python -u tools/kbench2d.py --dtype f32 > gpurun_out/r06/${T}_k2d_f32_g32pipe.txt 2>&1 || exit 7
echo "== g32pipe"; grep -E "^(FA|FB|I|Z4|T|B|S) " gpurun_out/r06/${T}_k2d_f32_g32pipe.txt; echo "== prod"; grep -E "^(T|B|S) " gpurun_out/r06/${T}_k2d_f32.txt
TAG=${T} bash tools/gpu_ab.sh "valu|DAMVS_X=1|--dtype f32" "mfma|DAMVS_PROB_MFMA=1|--dtype f32" "valu2|DAMVS_X=1|--dtype f32" "mfma2|DAMVS_PROB_MFMA=1|--dtype f32"
