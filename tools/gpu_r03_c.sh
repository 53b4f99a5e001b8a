#!/usr/bin/env bash
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
bash tools/vmcnt_probe/run.sh > gpurun_out/vmcnt_probe.log 2>&1 && echo "vmcnt probe done" && cat gpurun_out/vmcnt_probe.json &&
DAMVS_WARP_NO_PIPE=1 DAMVS_LIB=damvsnet_amd/ab/libdamvs_diaglds.so timeout -k 10 300 python -u tools/diag_streams2.py 0 1 7 > gpurun_out/diag2_lds_nopipe.log 2>&1 && echo "lds nopipe done" &&
grep -o '"layer": "[^"]*", "trials": [0-9]*, "outputs": [0-9]*, "differ_kernel_compare": [0-9]*' gpurun_out/diag2_lds_nopipe.log
