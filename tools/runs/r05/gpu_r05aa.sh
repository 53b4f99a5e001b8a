#!/bin/bash
# Round-5 aa: the wide conv2d kernel skipping the MFMAs of N-groups past the q-grid in partial column tiles --
# front-end layer times against the previous build (ab/libdamvs_pk.so: same conv2d sources as HEAD~1), then the
# front-end and stream tests on the new build.
mkdir -p gpurun_out/r05aa; O=gpurun_out/r05aa
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return $rc; }
for dt in bf16 f32; do for v in pk prod; do
  L=damvsnet_amd/libdamvs.so; [ $v = pk ] && L=damvsnet_amd/ab/libdamvs_pk.so
  DAMVS_LIB=$L step timeout -k 10 200 python -u tools/layer_times.py --dtype $dt --top 60 > $O/layers_${v}_$dt.txt 2>&1
  echo "$v $dt: $(grep 'per group (ms)' $O/layers_${v}_$dt.txt)"
done; done
step timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_frontend.py tests/test_gpu_streams.py > $O/pytest_frontend_streams.log 2>&1
tail -2 $O/pytest_frontend_streams.log
exit 0
