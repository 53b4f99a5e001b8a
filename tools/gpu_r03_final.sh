#!/usr/bin/env bash
# round-3 end refresh: full GPU suite, bf16 headline bench (with the CPU baseline), fp32 bench line, rocprofv3 stats of
# the default bench (roofline kernel check), one-stream per-kernel step table, in-pipeline warp PMC (traffic) and
# MFMA-utilisation PMC of the current kernels
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/pytest_gpu_z.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu_z.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_z.json 2> gpurun_out/bench_z.err || { tail -3 gpurun_out/bench_z.err; exit 1; }
tail -1 gpurun_out/bench_z.json | cut -c1-300
timeout -k 10 300 python -u bench.py --dtype f32 --no-cpu-baseline > gpurun_out/bench_f32_z.json 2> gpurun_out/bench_f32_z.err || { tail -3 gpurun_out/bench_f32_z.err; exit 1; }
tail -1 gpurun_out/bench_f32_z.json | cut -c1-200
timeout -k 10 600 python -u tools/pmc_warp_inpipe.py --out gpurun_out/pmc_inpipe_z > gpurun_out/pmc_inpipe_z.log 2>&1 || { tail -5 gpurun_out/pmc_inpipe_z.log; exit 1; }
timeout -k 10 300 python -u tools/pmc_mfma.py --out gpurun_out/pmcm_z > gpurun_out/pmc_mfma_z.log 2>&1 || { tail -5 gpurun_out/pmc_mfma_z.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_default -o run -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/prof_default_z.log" 2>&1 || { tail -3 "$R/gpurun_out/prof_default_z.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_q -o run -- python3 "$R/bench.py" --streams 1 --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/prof_q_z.log" 2>&1 || { tail -3 "$R/gpurun_out/prof_q_z.log"; exit 1; }
cd "$R" && cp /tmp/prof_default/run_kernel_stats.csv gpurun_out/bench_default_kernel_stats_z.csv && \
  python tools/prof_roofline_kernel.py /tmp/prof_default/run_kernel_trace.csv > gpurun_out/roofline_check_z.txt && \
  grep '^{"metric"' gpurun_out/prof_default_z.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench line (under rocprofv3): value %s, roofline ms_per_launch %s, isolated_ms_per_launch %s" % (d["value"], d["roofline"]["ms_per_launch"], d["roofline"]["isolated_ms_per_launch"]))' >> gpurun_out/roofline_check_z.txt && \
  python tools/prof_steps.py /tmp/prof_q/run_kernel_trace.csv 2 5 60 > gpurun_out/steps_z.txt && cat gpurun_out/roofline_check_z.txt && head -3 gpurun_out/steps_z.txt
