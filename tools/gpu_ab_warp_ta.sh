#!/bin/bash
# Warp gather-bound A/B (diagnostic builds, wrong results): the product library against SAMEX (east corners re-read the
# west ones: same loads, half the distinct lines) and 2TAP (west corners only: half the loads), stages 1-3, cfgC B=4,
# bf16 and fp32. Build first: tools/build_variant.sh samex -DDAMVS_DIAG_WARP_SAMEX; ... twotap -DDAMVS_DIAG_WARP_2TAP
mkdir -p gpurun_out
out=gpurun_out/ab_warp_ta.txt; : > $out
for lib in "" damvsnet_amd/ab/libdamvs_samex.so damvsnet_amd/ab/libdamvs_twotap.so; do
  for dt in bf16 f32; do
    for s in 1 2 3; do
      echo -n "${lib:-product} " >> $out
      DAMVS_LIB=$lib timeout -k 10 120 python -u tools/kbench.py --kernel warp --stage $s --batch 4 --dtype $dt --iters 10 >> $out 2>/dev/null || exit $?
    done
  done
done
cat $out
