#!/usr/bin/env bash
# the nontemporal-store volume write (-DDAMVS_DIAG_WARP_NT=1) against the same build plus an
# agent-scope release fence at the warp kernels' end (-DDAMVS_DIAG_WARP_NT_RELEASE=1), on the 2- and 4-stream
# bitwise tests (tools/build_variant.sh nt / ntrel). A failing variant is a result, not an error: every run is
# recorded in gpurun_out/${TAG}_nt.txt; the script stops only on a crash or time limit.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
TAG="${TAG:-nt}"
out=gpurun_out/${TAG}_nt.txt
: > $out
for v in nt ntrel; do
  DAMVS_LIB=damvsnet_amd/ab/libdamvs_$v.so timeout -k 10 400 python -u -m pytest -x -v -p no:cacheprovider \
    --timeout 240 --timeout-method thread tests/test_gpu_streams.py > gpurun_out/${TAG}_nt_$v.log 2>&1; rc=$?
  echo "$v rc=$rc $(grep -cE 'PASSED' gpurun_out/${TAG}_nt_$v.log) passed $(grep -cE 'FAILED' gpurun_out/${TAG}_nt_$v.log) failed" | tee -a $out
  grep -E "AssertionError|assert " gpurun_out/${TAG}_nt_$v.log | head -5 >> $out
  # 0 = pass, 1 = a bitwise mismatch (the experiment's possible outcome); anything else ends the call
  [ $rc -le 1 ] || exit $rc
done
exit 0
