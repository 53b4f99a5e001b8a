#!/bin/bash
# Round-5 q: MFMA utilisation per kernel family (tools/pmc_mfma.py), bf16 and fp32, on the final code.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r05q; mkdir -p $O
for dt in bf16 f32; do
  timeout -k 10 900 python -u tools/pmc_mfma.py --dtype $dt --out $O --tmp gpurun_out/pmc_mfma_$dt > $O/pmc_mfma_$dt.log 2>&1; rc=$?
  tail -c 1200 $O/pmc_mfma_$dt.log; rm -rf gpurun_out/pmc_mfma_$dt; [ $rc -ne 0 ] && exit $rc
done
exit 0
