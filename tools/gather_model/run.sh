#!/usr/bin/env bash
# build + run the gather cost model (L1-resident and L2-resident regions)
set -eu
D="$(cd "$(dirname "$0")" && pwd)"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o "$D/gather_model" "$D/gather_model.hip"
timeout -k 5 60 "$D/gather_model" 16384
timeout -k 5 60 "$D/gather_model" 262144
timeout -k 5 60 "$D/gather_model" 4194304
