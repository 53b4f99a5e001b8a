#!/usr/bin/env bash
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
DAMVS_LIB=damvsnet_amd/ab/libdamvs_diaglds.so timeout -k 10 300 python -u tools/diag_streams2.py 0 7 > gpurun_out/diag2_lds_shape.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids gpurun_out/diag2_lds_shape.log | cut -c1-3000
