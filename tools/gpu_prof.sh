#!/bin/bash
# rocprofv3 kernel trace of a short bench; per-launch table of the last step -> gpurun_out/launches.txt
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_q -o run -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_q.log 2>&1 || exit $?
cd $R && python tools/prof_damvs_launches.py gpurun_out/prof_q/run_kernel_trace.csv 4 > gpurun_out/launches.txt && python tools/prof_steps.py gpurun_out/prof_q/run_kernel_trace.csv > gpurun_out/steps.txt && head -3 gpurun_out/steps.txt
