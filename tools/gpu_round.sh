#!/bin/bash
# One GPU-box pass: parity tests, full bench (with CPU baseline), PMC traffic of the roofline kernel,
# rocprofv3 kernel trace of a short bench. Every GPU step has its own time limit; stops at the first
# fault/abort/timeout (exit codes > 1).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -20
[ $rc -le 1 ] || exit $rc
# PMC pass first (bench.py reads the per-launch HBM bytes from profiles/r01 at its batch)
timeout -k 10 400 python tools/pmc_traffic.py --kernel warp --stage 2 --config cfgC --batch 4 --out $R/profiles/r01 > gpurun_out/pmc_traffic.log 2>&1; rc=$?
echo "pmc rc=$rc"; tail -2 gpurun_out/pmc_traffic.log
[ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/profiles_new && cp $R/profiles/r01/pmc_*_b4.json gpurun_out/profiles_new/
timeout -k 10 500 python bench.py > gpurun_out/bench_full.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench_full.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_last -o run -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_last.log 2>&1; rc=$?
echo "prof rc=$rc"
exit $rc
