#!/bin/bash
# 1) rocprofv3 kernel trace + stats of the default bench command (timed steps on 2 streams, attribution
#    pass on one): stats CSV, its bench line, and the roofline kernel's per-grid means (roofline_check.txt);
# 2) the same with --streams 1 for the per-step kernel table (steps.txt) and per-launch table (launches.txt).
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_default -o run -- python $R/bench.py --no-cpu-baseline > $R/gpurun_out/prof_default.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_q -o run -- python $R/bench.py --streams 1 --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_q.log 2>&1 || exit $?
cd $R && python tools/prof_roofline_kernel.py gpurun_out/prof_default/run_kernel_trace.csv > gpurun_out/roofline_check.txt && \
  grep '^{"metric"' gpurun_out/prof_default.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench line (under rocprofv3): value %s, roofline ms_per_launch %s, isolated_ms_per_launch %s" % (d["value"], d["roofline"]["ms_per_launch"], d["roofline"]["isolated_ms_per_launch"]))' >> gpurun_out/roofline_check.txt && \
  python tools/prof_damvs_launches.py gpurun_out/prof_q/run_kernel_trace.csv 4 > gpurun_out/launches.txt && \
  python tools/prof_steps.py gpurun_out/prof_q/run_kernel_trace.csv > gpurun_out/steps.txt && cat gpurun_out/roofline_check.txt && head -3 gpurun_out/steps.txt
