#!/usr/bin/env bash
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
bash tools/gpu_r03_diag2.sh && bash tools/gpu_r03_order.sh
