#!/bin/bash
# Round-5 n (diagnostic): the failing fv3 warp (explicit-FMA sample coordinate) built plain (fv3pad0) and with an s_nop
# before every instruction of k_warp.hip (fv3pad1, -mllvm -amdgpu-snop-padding=1), through DAMVS_LIB.
mkdir -p gpurun_out
for v in fv3pad0 fv3pad1; do
  DAMVS_LIB=damvsnet_amd/ab/libdamvs_$v.so timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_streams.py > gpurun_out/r05n_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 gpurun_out/r05n_$v.log)"; [ $rc -ge 124 ] && exit $rc
done
exit 0
