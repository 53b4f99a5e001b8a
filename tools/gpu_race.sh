#!/usr/bin/env bash
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
for L in ${@:-unet regress 0 1 2 3 4 5 6 7 8 9}; do
  RACE_LAYER=$L timeout -k 10 120 python tools/streams_race_kernel.py > gpurun_out/rk_$L.log 2>&1 || { tail -3 gpurun_out/rk_$L.log; exit 1; }
  grep "RACE_LAYER" gpurun_out/rk_$L.log
done
