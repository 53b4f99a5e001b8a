#!/usr/bin/env bash
# MFMA prob conv + regression by default for bf16: full GPU suite, then bench x2 and the per-kernel step profile
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu_m.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu_m.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_m_$rep.json 2> gpurun_out/bench_m_$rep.err || { tail -3 gpurun_out/bench_m_$rep.err; exit 1; }
  python - "gpurun_out/bench_m_$rep.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("maps/s", d["value"], "ms/stage", d["ms_per_stage"], flush=True)
PY
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_q -o run -- python3 "$R/bench.py" --streams 1 --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/prof_q_m.log" 2>&1 || { tail -5 "$R/gpurun_out/prof_q_m.log"; exit 1; }
cd "$R" && python tools/prof_steps.py /tmp/prof_q/run_kernel_trace.csv 2 5 60 > gpurun_out/steps_m.txt && head -25 gpurun_out/steps_m.txt
