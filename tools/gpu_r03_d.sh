#!/usr/bin/env bash
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
summ() { grep -o '"layer": "[^"]*", "trials": [0-9]*, "outputs": [0-9]*, "differ_kernel_compare": [0-9]*' "$1"; }
timeout -k 10 120 tools/vmcnt_probe/vmcnt_deep > gpurun_out/vmcnt_deep.json 2> gpurun_out/vmcnt_deep.err && cat gpurun_out/vmcnt_deep.json &&
DAMVS_LIB=damvsnet_amd/ab/libdamvs_diagldsfw.so timeout -k 10 300 python -u tools/diag_streams2.py 0 1 7 > gpurun_out/diag2_lds_fullwait.log 2>&1 && echo "lds fullwait:" && summ gpurun_out/diag2_lds_fullwait.log &&
DIAG_TRIALS=12 timeout -k 10 400 python -u tools/diag_streams2.py 0 1 7 > gpurun_out/diag2_prod_heavy.log 2>&1 && echo "product heavy:" && summ gpurun_out/diag2_prod_heavy.log
