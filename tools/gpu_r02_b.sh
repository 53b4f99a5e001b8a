#!/usr/bin/env bash
# Round 2: full GPU suite, bench (in-pipeline roofline), sharded rehearsal, MFMA PMC pass.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_cfgC.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_cfgC.log; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config cfgD --shard depth --emulate 4 --steps 3 --warmup 1 > gpurun_out/bench_shard.log 2>&1; rc=$?
echo "shard rc=$rc"; tail -c 1500 gpurun_out/bench_shard.log; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/pmc_mfma.py --config cfgC --batch 4 --out gpurun_out/profiles_r02 > gpurun_out/pmc_mfma.log 2>&1; rc=$?
echo "pmc rc=$rc"; tail -c 2000 gpurun_out/pmc_mfma.log
exit $rc
