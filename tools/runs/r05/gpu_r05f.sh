#!/bin/bash
# Round-5 profile f: rocprofv3 kernel trace + stats of the default bench command (tools/gpu_prof.sh), then a one-stream
# fp32 bench under the kernel trace for the per-step kernel table of the parity path (steps_f32.txt).
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
bash $R/tools/gpu_prof.sh || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_f32 -o run -- python $R/bench.py --dtype f32 --streams 1 --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_f32.log 2>&1 || exit $?
cd $R && python tools/prof_steps.py gpurun_out/prof_f32/run_kernel_trace.csv 2 5 60 > gpurun_out/steps_f32.txt && head -3 gpurun_out/steps_f32.txt
