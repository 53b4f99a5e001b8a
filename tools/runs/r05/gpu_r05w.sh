#!/bin/bash
# Round-5 w (diagnostic): the failing fv3 warp (explicit-FMA sample coordinate) built without packed-FP32 VALU ops
# (fv3noslp: -fno-slp-vectorize for the warp unit, no v_pk_*_f32 left) and with its per-sample reciprocal on FMAs
# instead of v_rcp_f32 (fv3nr): the stream tests and the wave-level diagnosis beside conv1.
mkdir -p gpurun_out/r05w
for v in fv3noslp fv3nr; do
  DAMVS_LIB=damvsnet_amd/ab/libdamvs_$v.so timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_streams.py > gpurun_out/r05w/pytest_$v.log 2>&1; rc=$?
  echo "$v streams: $(tail -1 gpurun_out/r05w/pytest_$v.log)"; [ $rc -ge 124 ] && exit $rc
  for dt in f32 bf16; do
    DAMVS_LIB=damvsnet_amd/ab/libdamvs_$v.so timeout -k 10 200 python -u tools/diag_warp_streams.py --layout nhwc --layer 1 --dtype $dt --stage 1 > gpurun_out/r05w/${v}_$dt.jsonl 2>gpurun_out/r05w/${v}_$dt.err || { tail -3 gpurun_out/r05w/${v}_$dt.err; exit 1; }
    echo "$v $dt: $(grep -c wave_analysis gpurun_out/r05w/${v}_$dt.jsonl) bad launches"
  done
done
exit 0
