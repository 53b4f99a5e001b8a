#!/bin/bash
# Round-5 k: (1) the product build's stream tests and conv parity tests (the fp32 stage-3 conv0 prefetch), then
# (2, diagnostic) the stream-hazard warp variants through DAMVS_LIB -- the shared-taps + explicit-FMA warp that failed
# the stream tests (libdamvs_sharedfma.so) and the same with the weight-net coefficients taken from SGPRs instead of
# per-lane kernarg loads (libdamvs_kqsgpr.so).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_parity.py -k "streams or sub_batches or conv0 or costregnet or warp" > gpurun_out/r05k_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r05k_pytest.log; [ $rc -ge 124 ] && exit $rc
for v in kqsgpr sharedfma; do
  DAMVS_LIB=damvsnet_amd/ab/libdamvs_$v.so timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_streams.py -k warp_beside > gpurun_out/r05k_$v.log 2>&1
  rc=$?; echo "$v rc=$rc: $(tail -1 gpurun_out/r05k_$v.log)"; [ $rc -ge 124 ] && exit $rc
done
exit 0
