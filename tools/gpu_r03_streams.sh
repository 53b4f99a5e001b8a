#!/usr/bin/env bash
# sub-batch stream count A/B with the round-3 kernels (bench --streams 1 / 2 / 4), two rounds
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
for st in 2 1 4 2 1 4; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 3 --streams $st > gpurun_out/bench_st.json 2> gpurun_out/bench_st.err || { echo "bench streams $st failed"; tail -3 gpurun_out/bench_st.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_st.json').read().strip().splitlines()[-1]); print(json.dumps({'streams': $st, 'maps_s': d['value'], 'ms_per_step': d['ms_per_step']}))" | tee -a gpurun_out/ab_streams.jsonl
done
