#!/bin/bash
# Round-6: sub-batch streams for the fp32 parity path (1 / 2 / 4 streams at B = 4) and the bf16 line at 4 streams.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06p}
TAG=${T} bash tools/gpu_ab.sh "f32 s2|DAMVS_X=1|--dtype f32" "f32 s4|DAMVS_X=1|--dtype f32 --streams 4" "f32 s1|DAMVS_X=1|--dtype f32 --streams 1" "f32 s4b|DAMVS_X=1|--dtype f32 --streams 4" "f32 s2b|DAMVS_X=1|--dtype f32" "bf16 s4|DAMVS_X=1|--no-parity-path --streams 4" "bf16 s2|DAMVS_X=1|--no-parity-path"
