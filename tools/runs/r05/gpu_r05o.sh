#!/bin/bash
# Round-5 o: the round's PMC inputs on the final code -- MFMA utilisation per kernel family and
# the in-pipeline stage-2 warp counters, bf16 and fp32 -- then the rocprofv3 kernel trace + stats of the default bench
# command (tools/gpu_prof.sh). Summaries land in gpurun_out/r05o/; the raw per-pass CSVs are deleted once summarised
# (gpurun copies back at most 64 MiB).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r05o; mkdir -p $O
for dt in bf16 f32; do
  echo "pmc_mfma $dt"; timeout -k 10 900 python -u tools/pmc_mfma.py --dtype $dt --out $O --tmp gpurun_out/pmc_mfma_$dt > $O/pmc_mfma_$dt.log 2>&1; rc=$?
  tail -c 1500 $O/pmc_mfma_$dt.log; rm -rf gpurun_out/pmc_mfma_$dt; [ $rc -ge 124 ] && exit $rc
  echo "pmc_warp_inpipe $dt"; PMC_DTYPE=$dt timeout -k 10 1200 python -u tools/pmc_warp_inpipe.py --out gpurun_out/pmc_inpipe_$dt > $O/pmc_inpipe_$dt.log 2>&1; rc=$?
  cp gpurun_out/pmc_inpipe_$dt/pmc_warp_inpipe.json $O/pmc_warp_inpipe_$dt.json 2>/dev/null; rm -rf gpurun_out/pmc_inpipe_$dt
  tail -3 $O/pmc_inpipe_$dt.log; [ $rc -ge 124 ] && exit $rc
done
echo "gpu_prof"; bash tools/gpu_prof.sh; rc=$?
for f in prof_default/run_kernel_stats.csv roofline_check.txt launches.txt steps.txt prof_default.log; do cp gpurun_out/$f $O/$(echo $f | tr / _) 2>/dev/null; done
rm -rf gpurun_out/prof_default gpurun_out/prof_q
exit $rc
