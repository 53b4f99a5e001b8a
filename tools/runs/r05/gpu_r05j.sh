#!/bin/bash
# Round-5 j: shared-taps warp (runtime view loop) + branch-free conv0 walk: their parity and stream tests, then warp and
# conv0 times against the HEAD build (damvsnet_amd/ab/libdamvs_base.so, tools/build_ab.sh).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_streams.py -k "warp or conv0 or costregnet or streams or sub_batches" > gpurun_out/r05j_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r05j_pytest.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/r05j_ab.txt; : > $out
for lib in damvsnet_amd/ab/libdamvs_base.so ""; do
  for dt in f32 bf16; do
    for s in 1 2 3; do
      echo -n "${lib:-new} " >> $out
      DAMVS_LIB=$lib timeout -k 10 120 python -u tools/kbench.py --kernel warp --stage $s --batch 4 --dtype $dt --iters 10 >> $out 2>/dev/null || exit $?
    done
    echo "${lib:-new}" >> $out
    DAMVS_LIB=$lib timeout -k 10 200 python -u tools/unet_layers.py --dtype $dt --only conv0 2>/dev/null | grep conv0 >> $out || exit $?
  done
done
cat $out
