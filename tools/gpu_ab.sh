#!/usr/bin/env bash
# A/B bench lines in one GPU call: each argument is "label|ENV=V ENV2=V2|bench args"; every variant runs as its own
# bench process (20 steps, 3 warm-up, no CPU baseline) under its own time limit, and its line (value, ms_per_step, the
# hot-path per-stage ms and the parity_path value) goes to gpurun_out/${TAG}_ab.jsonl. Stops at the first failure.
#   TAG=r04h tools/gpu_ab.sh "bf16 fused|DAMVS_HEAD_FUSE=1|--no-parity-path" "bf16 split|DAMVS_HEAD_FUSE=0|--no-parity-path"
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
TAG="${TAG:-ab}"
out=gpurun_out/${TAG}_ab.jsonl
for spec in "$@"; do
  label="${spec%%|*}"; rest="${spec#*|}"; envs="${rest%%|*}"; args="${rest#*|}"
  env $envs timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline $args \
    > gpurun_out/${TAG}_ab_last.json 2> gpurun_out/${TAG}_ab_last.err; rc=$?
  [ $rc -eq 0 ] || { echo "$label rc=$rc"; tail -20 gpurun_out/${TAG}_ab_last.err; exit $rc; }
  tail -1 gpurun_out/${TAG}_ab_last.json | python -c '
import json, sys
d = json.loads(sys.stdin.read())
hp = {k: {g: v["kernels"][g]["ms"] for g in v["kernels"]} for k, v in d["hot_path_roofline"]["per_stage"].items()}
r = {"label": sys.argv[1], "env": sys.argv[2], "args": sys.argv[3], "value": d["value"], "ms_per_step": d["ms_per_step"],
     "dtype": d["dtype"], "hot": hp, "stages": d.get("ms_per_stage"), "parity_path": (d.get("parity_path") or {}).get("value")}
print(json.dumps(r))' "$label" "$envs" "$args" | tee -a $out
done
exit 0
