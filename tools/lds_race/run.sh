#!/usr/bin/env bash
# GPU step: build and run the LDS co-residency experiment (writes gpurun_out/lds_race.json).
set -eu
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
mkdir -p "$R/gpurun_out"
cd "$R/tools/lds_race"
[ -x lds_race ] || /opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 lds_race.hip -o lds_race
timeout -k 10 120 ./lds_race "${1:-8}" > "$R/gpurun_out/lds_race.json"
cat "$R/gpurun_out/lds_race.json"
