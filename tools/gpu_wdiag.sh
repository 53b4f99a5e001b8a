#!/usr/bin/env bash
# Time kbench2d case N with each wide-kernel knock-out build (tools/build_diag_wide.sh); timing only.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
for m in ${MASKS:-0 1 2 4 8 15}; do
  L=$R/damvsnet_amd/libdamvs.so; [ $m = 0 ] || L=$R/damvsnet_amd/ab/libdamvs_wdiag$m.so
  DAMVS_LIB=$L timeout -k 10 120 python -u tools/kbench2d.py --only N,F > gpurun_out/wd$m.log 2>&1 || { tail -3 gpurun_out/wd$m.log; exit 1; }
  echo "mask $m: $(grep -E '^(N|F) ' gpurun_out/wd$m.log | tr -s ' ' | cut -d' ' -f1,8-9 | tr '\n' ' ')"
done
