#!/usr/bin/env bash
# Checkpoint: full GPU suite; in-pipeline PMC of the stage-2 warp (copied into profiles/r02 so the bench line reports
# it as traffic); default bench line with the CPU baseline; cfgD / cfgE lines; rocprofv3 kernel-trace profiles.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -10
[ $rc -eq 0 ] || exit $rc
PMC_WARP_KERNEL="warp_aggregate_kernel<unsigned short, 16, 0, false" timeout -k 10 600 python -u tools/pmc_warp_inpipe.py \
  --out gpurun_out/pmc_inpipe > gpurun_out/pmc_inpipe.log 2>&1; rc=$?
echo "pmc rc=$rc"; tail -c 1500 gpurun_out/pmc_inpipe.log; echo
[ $rc -eq 0 ] || exit $rc
cp gpurun_out/pmc_inpipe/pmc_warp_inpipe.json profiles/r02/pmc_warp_inpipe_cfgC_b4.json
timeout -k 10 400 python -u bench.py > gpurun_out/bench_cfgC.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench_cfgC.log | cut -c1-300; echo
[ $rc -eq 0 ] || exit $rc
for c in cfgD cfgE; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1 || { tail -5 gpurun_out/bench_$c.log; exit 1; }
  grep '^{"metric"' gpurun_out/bench_$c.log | tail -1 > gpurun_out/bench_${c}_line.json
  echo "$c: $(cut -c1-120 gpurun_out/bench_${c}_line.json)"
done
bash tools/gpu_prof.sh
