#!/usr/bin/env bash
# A/B of the bf16 in-place skip epilogue variants (tools/diag_skip_epilogue.py) on the case that lost skip
# terms every run in round 1 (B=4, D=64, 64x160, stage-1 channels), deconvs on the gather kernel.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
for st in 1 0; do for v in 0 1 2 3 4; do
  lib=damvsnet_amd/libdamvs.so; [ $v -gt 0 ] && lib=damvsnet_amd/diag/libdamvs_skip$v.so
  echo "=== stage $st variant $v ($lib)"
  DAMVS_LIB=$lib DAMVS_DECONV_NO_ZSLIDE=1 DAMVS_CONV_NO_ZSLIDE=${NOZ:-0} timeout -k 10 120 python -u tools/diag_unet_repro.py --B 4 --D 64 --H 64 \
    --W 160 --stage $st --runs 8 > gpurun_out/diag_skip${st}_$v.log 2>&1; rc=$?
  grep -E "^run|  c[0-9]|logits:" gpurun_out/diag_skip${st}_$v.log | head -30
  [ $rc -eq 0 ] || exit $rc
done; done
