#!/bin/bash
# Round-5 v (diagnostic): which step of the sample-coordinate chain comes out different in lanes 48-63 -- the chain
# computed twice per sample (opaque hypothesis copies), a record carries the mask of differing intermediates
# (bit 0 qx, 1 qy, 2 qz, 3 1/qz, 4 ix, 5 iy, 6 first weight, 7 first offset).
mkdir -p gpurun_out/r05v
for dt in f32 bf16; do
  DAMVS_LIB=damvsnet_amd/ab/libdamvs_chkparts.so timeout -k 10 200 python -u tools/diag_warp_streams.py --layout nhwc --layer 1 --dtype $dt --stage 1 > gpurun_out/r05v/chkparts_$dt.jsonl 2>gpurun_out/r05v/chkparts_$dt.err || { tail -3 gpurun_out/r05v/chkparts_$dt.err; exit 1; }
  echo "chkparts $dt: $(grep -c wave_analysis gpurun_out/r05v/chkparts_$dt.jsonl) bad launches"
  grep diag_records gpurun_out/r05v/chkparts_$dt.jsonl | grep -v '"count": 0' | head -3 | cut -c1-600
done
exit 0
