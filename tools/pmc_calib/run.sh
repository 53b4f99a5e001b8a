#!/usr/bin/env bash
# GPU step: FETCH_SIZE calibration for gathers (calib.hip). Writes gpurun_out/pmc_calib/{calib_timing.jsonl, summary.json}.
set -eu
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R/tools/pmc_calib"
[ -x calib ] || /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 calib.hip -o calib
O="$R/gpurun_out/pmc_calib"; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 60 ./calib > "$O/calib_timing.jsonl"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$O/fetch" -o run -- "$R/tools/pmc_calib/calib" > "$O/prof_fetch.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum --kernel-trace --output-format csv -d "$O/rdreq" -o run -- "$R/tools/pmc_calib/calib" > "$O/prof_rdreq.log" 2>&1
python3 "$R/tools/pmc_calib/parse.py" "$O" > "$O/summary.json"
cat "$O/summary.json"
