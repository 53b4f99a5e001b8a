#!/bin/bash
# Round-5 check d: which variant of the fp32 warp / conv1 pair shows the lanes-48-63 corruption beside another stream.
mkdir -p gpurun_out
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return 0; }
run() {  # run <tag> <stage> [ENV=...]
  local tag=$1 st=$2; shift 2
  env "$@" timeout -k 10 120 python -u tools/diag_warp_streams.py --layout nhwc --layer 1 --dtype f32 --stage $st \
    > gpurun_out/r05d_$tag.jsonl 2>&1; rc=$?
  [ $rc -ge 124 ] && { echo "hard failure rc=$rc ($tag)"; exit $rc; }
  echo "$tag: $(grep -c '"voxels": 0' gpurun_out/r05d_$tag.jsonl) clean of $(grep -c voxels gpurun_out/r05d_$tag.jsonl)"
}
for st in 1 0; do
  run default_s$st $st X=1
  run onelane_s$st $st DAMVS_WARP_SPLIT=0
  run conv1gather_s$st $st DAMVS_DECONV_NO_ZSLIDE=1
  run norv_s$st $st DAMVS_WARP_RUNTIME_VIEWS=1
done
