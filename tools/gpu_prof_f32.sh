#!/bin/bash
# rocprofv3 kernel trace of the fp32 parity path on one stream (bench.py --dtype f32 --streams 1): the per-step kernel
# table (gpurun_out/<TAG>_steps_f32.txt).
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
T=${TAG:-prof_f32}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_q -o run -- python $R/bench.py --dtype f32 --streams 1 --steps 5 --warmup 2 --no-cpu-baseline --no-shard-latency > $R/gpurun_out/${T}_q.log 2>&1 || exit $?
cd $R && python tools/prof_steps.py gpurun_out/${T}_q/run_kernel_trace.csv > gpurun_out/${T}_steps_f32.txt && head -45 gpurun_out/${T}_steps_f32.txt
