#!/bin/bash
# Round-5 ac: bf16 wide conv2d with A fragments per wave from L1 / L2 (no LDS A copy, one barrier per 32-channel
# slice; ab/libdamvs_agb.so) against the product: front-end tests on the variant, then bf16 layer times, twice each.
mkdir -p gpurun_out/r05ac; O=gpurun_out/r05ac
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return $rc; }
DAMVS_LIB=damvsnet_amd/ab/libdamvs_agb.so step timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_frontend.py > $O/pytest_frontend_agb.log 2>&1
echo "agb frontend: $(tail -1 $O/pytest_frontend_agb.log)"
for r in 1 2; do for v in prod agb; do
  L=damvsnet_amd/libdamvs.so; [ $v = agb ] && L=damvsnet_amd/ab/libdamvs_agb.so
  DAMVS_LIB=$L step timeout -k 10 200 python -u tools/layer_times.py --dtype bf16 --top 60 > $O/layers_${v}_$r.txt 2>&1
  echo "$v run $r: $(grep 'per group (ms)' $O/layers_${v}_$r.txt)"
done; done
exit 0
