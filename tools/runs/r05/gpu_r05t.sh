#!/bin/bash
# Round-5 t (diagnostic): wave-level shape of the stream fault in the fv3 warp (explicit-FMA sample coordinate), NHWC
# maps, beside conv1 on another stream: fp32 and bf16 at stage 2, fp32 at stage 1.
mkdir -p gpurun_out/r05t
for args in "--dtype f32 --stage 1" "--dtype bf16 --stage 1" "--dtype f32 --stage 0"; do
  tag=$(echo $args | tr -d ' -')
  DAMVS_LIB=damvsnet_amd/ab/libdamvs_fv3.so timeout -k 10 200 python -u tools/diag_warp_streams.py --layout nhwc --layer 1 $args > gpurun_out/r05t/$tag.jsonl 2>gpurun_out/r05t/$tag.err || { tail -3 gpurun_out/r05t/$tag.err; exit 1; }
  grep -c wave_analysis gpurun_out/r05t/$tag.jsonl
done
exit 0
