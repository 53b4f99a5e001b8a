#!/usr/bin/env bash
set -eu
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R/tools/vmcnt_probe"
[ -x vmcnt_probe ] || /opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 vmcnt_probe.hip -o vmcnt_probe
mkdir -p "$R/gpurun_out"
timeout -k 10 120 ./vmcnt_probe > "$R/gpurun_out/vmcnt_probe.json"
cat "$R/gpurun_out/vmcnt_probe.json"
