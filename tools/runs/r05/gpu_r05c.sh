#!/bin/bash
# Round-5 check c: the fp32 warp beside conv1 on another stream (default vs clamp build), the stream tests on the clamp
# build, the range tests, and PMC of the wide rolling kernel (case N) against the previous loop.
mkdir -p gpurun_out
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return 0; }
for dt in f32 bf16; do for st in 1 0; do
  step timeout -k 10 120 python -u tools/diag_warp_streams.py --layout nhwc --layer 1 --dtype $dt --stage $st > gpurun_out/r05c_diag_${dt}_s${st}_l1.jsonl 2>&1
  DAMVS_LIB=damvsnet_amd/ab/libdamvs_clamp.so step timeout -k 10 120 python -u tools/diag_warp_streams.py --layout nhwc --layer 1 --dtype $dt --stage $st > gpurun_out/r05c_diag_${dt}_s${st}_l1_clamp.jsonl 2>&1
done; done
for f in gpurun_out/r05c_diag_*.jsonl; do echo "$f $(grep -c '"voxels": 0' $f) clean of $(grep -c voxels $f)"; done
DAMVS_LIB=damvsnet_amd/ab/libdamvs_clamp.so step timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread \
  tests/test_gpu_streams.py > gpurun_out/r05c_pytest_streams_clamp.log 2>&1
tail -3 gpurun_out/r05c_pytest_streams_clamp.log
step timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread "tests/test_gpu_parity.py::test_cascade_range_status_fp32" \
  "tests/test_gpu_parity.py::test_depthnet_range_status" > gpurun_out/r05c_pytest_range.log 2>&1
tail -2 gpurun_out/r05c_pytest_range.log
step timeout -k 10 500 bash tools/pmc_k2d.sh r05c_pmc_rs f32 N > gpurun_out/r05c_pmc_rs.txt 2>&1
cat gpurun_out/r05c_pmc_rs.txt | tail -8
DAMVS_WIDE_RS=0 step timeout -k 10 500 bash tools/pmc_k2d.sh r05c_pmc_ag f32 N > gpurun_out/r05c_pmc_ag.txt 2>&1
cat gpurun_out/r05c_pmc_ag.txt | tail -8
