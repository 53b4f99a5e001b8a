#!/bin/bash
# Round-6 checkpoint B: rocprofv3 kernel trace + stats of the default bench command (tools/gpu_prof.sh), then the MFMA
# utilisation PMC of both dtypes (tools/pmc_mfma.py) into gpurun_out/r06/pmc.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06/pmc
bash tools/gpu_prof.sh || exit 3
cd $R
for dt in bf16 f32; do
  timeout -k 10 600 python -u tools/pmc_mfma.py --config cfgC --batch 4 --dtype $dt --out $R/gpurun_out/r06/pmc --tmp $R/gpurun_out/pmc_mfma_$dt > gpurun_out/r06/pmc/pmc_mfma_$dt.log 2>&1 || { tail -5 gpurun_out/r06/pmc/pmc_mfma_$dt.log; exit 4; }
  tail -3 gpurun_out/r06/pmc/pmc_mfma_$dt.log
done
