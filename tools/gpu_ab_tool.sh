#!/bin/bash
# A/B of one per-layer tool across environments / library builds in one GPU call: each argument is
# "label|ENV=V ENV2=V2|tool args" (e.g. "s2 off|DAMVS_CONV2D_LDS_S2=0|tools/kbench2d.py --dtype f32 --only FA,FB";
# "head|DAMVS_LIB=damvsnet_amd/ab/libdamvs_base.so|tools/unet_layers.py --dtype f32 --only conv11"). Each variant runs
# as its own process under its own time limit; its output goes to gpurun_out/${TAG}_<n>.txt and its table lines to
# stdout. Stops at the first failure. (Round 6's one-off A/B scripts, tools/gpu_r06*.sh up to commit 0fa9d58, were all of
# this form or of tools/gpu_ab.sh's.)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
TAG="${TAG:-abtool}"
i=0
for spec in "$@"; do
  i=$((i+1))
  label="${spec%%|*}"; rest="${spec#*|}"; envs="${rest%%|*}"; args="${rest#*|}"
  env $envs timeout -k 10 300 python -u $args > gpurun_out/${TAG}_$i.txt 2>&1; rc=$?
  echo "== $label ($envs)"
  [ $rc -eq 0 ] || { echo "rc=$rc"; tail -20 gpurun_out/${TAG}_$i.txt; exit $rc; }
  grep -E " us | ms |valu|mfma" gpurun_out/${TAG}_$i.txt | grep -v "^\[" | head -60
done
exit 0
