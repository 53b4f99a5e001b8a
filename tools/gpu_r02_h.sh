#!/usr/bin/env bash
# Checkpoint: MFMA-utilisation PMC pass (copied into profiles/r02 so the bench line reports it), full GPU suite,
# default bench line (with the CPU baseline), kernel-trace profiles of the bench (tools/gpu_prof.sh).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u tools/pmc_mfma.py --config cfgC --batch 4 --out gpurun_out/profiles_r02 > gpurun_out/pmc_mfma.log 2>&1; rc=$?
echo "pmc rc=$rc"; tail -c 600 gpurun_out/pmc_mfma.log; echo
[ $rc -eq 0 ] || exit $rc
cp gpurun_out/profiles_r02/pmc_mfma_cfgC_b4.json profiles/r02/
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_cfgC.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench_cfgC.log | cut -c1-400; echo
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh
