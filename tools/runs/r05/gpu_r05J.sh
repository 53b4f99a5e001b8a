#!/bin/bash
# Round-5 J: halo conv2d with A fragments three chunks ahead (product) against HEAD (ab/libdamvs_base.so): narrow-layer
# microbench (bf16, fp32), front-end tests, per-layer times.
mkdir -p gpurun_out/r05J; O=gpurun_out/r05J
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return $rc; }
step timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_frontend.py > $O/pytest_frontend.log 2>&1
echo "frontend: $(tail -1 $O/pytest_frontend.log)"
for dt in bf16 f32; do for v in base prod; do
  L=damvsnet_amd/libdamvs.so; [ $v = base ] && L=damvsnet_amd/ab/libdamvs_base.so
  DAMVS_LIB=$L step timeout -k 10 200 python -u tools/kbench2d.py --dtype $dt --only G4,M4,Z4,T,O,P,Q,J,K,L,R --iters 20 > $O/kb2d_${v}_$dt.txt 2>&1
  echo "== $v $dt"; grep " us " $O/kb2d_${v}_$dt.txt | awk '{print $1, $(NF-5), $(NF-4)}' | tr '\n' ';'; echo
done; done
for dt in bf16 f32; do for v in base prod; do
  L=damvsnet_amd/libdamvs.so; [ $v = base ] && L=damvsnet_amd/ab/libdamvs_base.so
  DAMVS_LIB=$L step timeout -k 10 200 python -u tools/layer_times.py --dtype $dt --top 80 > $O/layers_${v}_$dt.txt 2>&1
  echo "$v $dt: $(grep 'per group (ms)' $O/layers_${v}_$dt.txt)"
done; done
exit 0
