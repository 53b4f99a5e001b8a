#!/usr/bin/env bash
# hyp_refine variants: parity suite (incl. the bitwise tests against one lane per pixel), then bench A/B of the
# stage hypotheses phases (DAMVS_HYP_QUAD=1: stage 2 with one lane per full-resolution point), three rounds
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/pytest_hyp.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_hyp.log; [ $rc -eq 0 ] || exit $rc
for v in X=1 DAMVS_HYP_QUAD=1 X=1 DAMVS_HYP_QUAD=1 X=1 DAMVS_HYP_QUAD=1; do
  env $v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { echo "bench $v failed"; tail -3 gpurun_out/bench_ab.err; exit 1; }
  python - "$v" gpurun_out/bench_ab.json <<'PY' | tee -a gpurun_out/ab_hyp.jsonl
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
m = d["ms_per_stage"]
print(json.dumps({"env": sys.argv[1], "maps_s": d["value"], "hypotheses_ms": [m["stage1.hypotheses"], m["stage2.hypotheses"], m["stage3.hypotheses"]]}), flush=True)
PY
done
