#!/usr/bin/env bash
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 120 tools/lds_race/lds_race2 > gpurun_out/lds_race2.json 2>&1; echo "rc=$?"; cat gpurun_out/lds_race2.json
