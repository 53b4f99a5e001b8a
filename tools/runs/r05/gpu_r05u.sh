#!/bin/bash
# Round-5 u (diagnostic): where the fault enters the fv3 warp -- builds that recompute every sample's taps with an
# opaque hypothesis (chktaps) or re-issue every gather with opaque offsets (chkloads) and append a record on any
# mismatch, beside conv1 on another stream (fp32 and bf16 stage 2); chk0: the same build without checks.
mkdir -p gpurun_out/r05u
for v in chk0 chktaps chkloads; do
  for dt in f32 bf16; do
    DAMVS_LIB=damvsnet_amd/ab/libdamvs_$v.so timeout -k 10 200 python -u tools/diag_warp_streams.py --layout nhwc --layer 1 --dtype $dt --stage 1 > gpurun_out/r05u/${v}_$dt.jsonl 2>gpurun_out/r05u/${v}_$dt.err || { tail -3 gpurun_out/r05u/${v}_$dt.err; exit 1; }
    echo "$v $dt: $(grep -c wave_analysis gpurun_out/r05u/${v}_$dt.jsonl) bad launches; $(grep diag_records gpurun_out/r05u/${v}_$dt.jsonl | grep -v '"count": 0' | head -2 | cut -c1-300)"
  done
done
exit 0
