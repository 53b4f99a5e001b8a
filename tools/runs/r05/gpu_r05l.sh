#!/bin/bash
# Round-5 l (diagnostic): bisect the explicit-FMA projection change that reopened the stream fault -- fv1: rays as FMAs,
# fv2: the depth step q = r hyp + t as an FMA, fv3: the sample coordinate as an FMA (each alone on the pinned warp).
mkdir -p gpurun_out
for v in fv1 fv2 fv3; do
  DAMVS_LIB=damvsnet_amd/ab/libdamvs_$v.so timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_streams.py -k warp_beside > gpurun_out/r05l_$v.log 2>&1
  rc=$?; echo "$v rc=$rc: $(tail -1 gpurun_out/r05l_$v.log)"; [ $rc -ge 124 ] && exit $rc
done
exit 0
