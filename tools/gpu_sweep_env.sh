#!/usr/bin/env bash
# Kernel-selection switch sweep (DESIGN.md section 4 switch table): every variant runs twice, each time
# right after a default run, so drift and run-to-run spread show up beside the deltas. B=4, 20 steps.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
run() {  # run <label> [VAR=value ...]
  local label=$1; shift
  env "$@" timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-shard-latency \
    > gpurun_out/sw.log 2>&1 || { echo "$label failed"; tail -3 gpurun_out/sw.log; exit 1; }
  echo "$label $(tail -1 gpurun_out/sw.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for cfg in "DAMVS_PROB_MFMA=0" "DAMVS_CONV_XPAIR=0" "DAMVS_CONV2D_XPAIR=0" "DAMVS_CONV_NO_ZSLIDE=1" \
           "DAMVS_DECONV_NO_ZSLIDE=1" "DAMVS_WIDE_RS=0" "DAMVS_HALO_RS=0" "DAMVS_CONV2D_G32=0"; do
  for rep in 1 2; do
    run "default" X=1
    run "$cfg" "$cfg"
  done
done
