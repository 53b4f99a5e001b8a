#!/usr/bin/env bash
# Round-3 concurrent-stream diagnosis, step 2: how the warp's outputs differ (sentinel-filled outputs, host vs
# kernel comparison, cache scrub), for the LDS-camera diag build and the product library.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
DAMVS_LIB=damvsnet_amd/ab/libdamvs_diaglds.so timeout -k 10 300 python -u tools/diag_streams2.py > gpurun_out/diag2_lds.log 2>&1 && echo "diag2 lds done" &&
timeout -k 10 300 python -u tools/diag_streams2.py > gpurun_out/diag2_prod.log 2>&1 && echo "diag2 prod done"
timeout -k 10 300 python -u tools/diag_bf16_error.py > gpurun_out/diag_bf16_error.log 2>&1 && echo "bf16 error done"
bash tools/pmc_calib/run.sh > gpurun_out/pmc_calib.log 2>&1 && echo "pmc calib done"
