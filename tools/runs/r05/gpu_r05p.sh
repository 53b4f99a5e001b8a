#!/bin/bash
# Round-5 p: unblocked NHWC against channel-blocked feature maps for the stage-1 warp (fp32: 128-byte pixels, the
# channel-split kernel at odd N, the one-lane kernel at even N; bf16: 64-byte pixels), cfgC B=4.
mkdir -p gpurun_out; out=gpurun_out/ab_warp_layout_r05p.txt; : > $out
for dt in f32 bf16; do
  for n in 5 6; do
    for lay in nhwc cblock; do
      timeout -k 10 120 python -u tools/kbench.py --kernel warp --stage 1 --batch 4 --dtype $dt --views $n --layout $lay --iters 10 >> $out 2>/dev/null || exit $?
    done
  done
done
cat $out
