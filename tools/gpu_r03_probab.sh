#!/usr/bin/env bash
# prob_mfma A/B: weight terms (3 / 2) x plane prefetch depth (4 / 3 / 6), isolated at the three cfgC stages (B=4)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
for v in default t2a4 t3a3 t2a3 t3a6; do
  lib=""; [ $v != default ] && lib="$R/damvsnet_amd/ab/libdamvs_$v.so"
  DAMVS_LIB=$lib timeout -k 10 200 python -u tools/kbench_prob.py > gpurun_out/probab_$v.jsonl 2>&1 || { tail -3 gpurun_out/probab_$v.jsonl; exit 1; }
  echo "$v: $(grep '"mfma", "prob_write": true' gpurun_out/probab_$v.jsonl | python -c 'import json,sys; print([json.loads(l)["ms"] for l in sys.stdin])')"
done
