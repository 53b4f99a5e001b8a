#!/usr/bin/env bash
# rocprofv3 kernel trace + stats of the default bench (2 streams) and of a one-stream run (per-step table);
# raw traces stay under /tmp, summaries go to gpurun_out; then the front-end per-layer table.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_default -o run -- python $R/bench.py --no-cpu-baseline > $R/gpurun_out/prof_default.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_q -o run -- python $R/bench.py --streams 1 --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_q.log 2>&1 || exit $?
cd $R && cp /tmp/prof_default/run_kernel_stats.csv gpurun_out/bench_default_kernel_stats.csv && \
  python tools/prof_roofline_kernel.py /tmp/prof_default/run_kernel_trace.csv > gpurun_out/roofline_check.txt && \
  grep '^{"metric"' gpurun_out/prof_default.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench line (under rocprofv3): value %s, roofline ms_per_launch %s, isolated_ms_per_launch %s" % (d["value"], d["roofline"]["ms_per_launch"], d["roofline"]["isolated_ms_per_launch"]))' >> gpurun_out/roofline_check.txt && \
  python tools/prof_steps.py /tmp/prof_q/run_kernel_trace.csv 2 5 60 > gpurun_out/steps.txt && cat gpurun_out/roofline_check.txt && head -3 gpurun_out/steps.txt &&
timeout -k 10 200 python tools/layer_times.py --top 70 > gpurun_out/layer_times.txt 2>&1 && head -2 gpurun_out/layer_times.txt
