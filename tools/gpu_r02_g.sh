#!/usr/bin/env bash
# block_channels repack parity, warp/stage subset; bench A/B over the number of concurrent sub-batch streams;
# one-stream rocprofv3 kernel table of the default bench (per-step table, per-launch table).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "block_channels or warp or stage or streams" > gpurun_out/pytest_g.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_g.log | tail -8
[ $rc -eq 0 ] || exit $rc
for st in 2 3 4 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --streams $st --steps 20 > gpurun_out/bench_st.log 2>&1 || { tail -5 gpurun_out/bench_st.log; exit 1; }
  echo "streams=$st: $(grep '^{"metric"' gpurun_out/bench_st.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["ms_per_stage"])')"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_q -o run -- python $R/bench.py --streams 1 --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_q.log 2>&1 || exit $?
cd $R && python tools/prof_damvs_launches.py gpurun_out/prof_q/run_kernel_trace.csv 4 > gpurun_out/launches.txt && \
  python tools/prof_steps.py gpurun_out/prof_q/run_kernel_trace.csv > gpurun_out/steps.txt && head -3 gpurun_out/steps.txt
