#!/usr/bin/env bash
# Round-3 concurrent-stream diagnosis: LDS co-residency experiment, the LDS-camera warp
# beside every U-Net layer with in-kernel records, the nontemporal-store warp under the stream tests.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 150 bash tools/lds_race/run.sh 16 > gpurun_out/lds_race.log 2>&1 && echo "lds_race done" &&
DAMVS_LIB=damvsnet_amd/ab/libdamvs_diaglds.so timeout -k 10 420 python -u tools/diag_streams.py > gpurun_out/diag_streams.log 2>&1 && echo "diag_streams done" &&
DAMVS_LIB=damvsnet_amd/ab/libdamvs_diagnt.so timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_streams.py > gpurun_out/pytest_nt.log 2>&1; echo "nt pytest rc=$?"
tail -5 gpurun_out/pytest_nt.log
