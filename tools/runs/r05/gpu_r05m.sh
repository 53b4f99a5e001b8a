#!/bin/bash
# Round-5 m: CU-exclusive warp blocks. (1) the product build's warp parity and stream tests; (2) the two instruction
# streams that failed the stream tests on shared CUs (xfv3: explicit-FMA sample coordinate; xshared: shared-taps view
# loop), now CU-exclusive, through DAMVS_LIB; (3) warp times: product vs the HEAD build (libdamvs_base.so) vs xshared.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_parity.py -k "streams or sub_batches or warp" > gpurun_out/r05m_pytest.log 2>&1
rc=$?; echo "product: $(tail -1 gpurun_out/r05m_pytest.log)"; [ $rc -ge 124 ] && exit $rc
for v in xfv3 xshared; do
  DAMVS_LIB=damvsnet_amd/ab/libdamvs_$v.so timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_streams.py > gpurun_out/r05m_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 gpurun_out/r05m_$v.log)"; [ $rc -ge 124 ] && exit $rc
done
out=gpurun_out/r05m_ab.txt; : > $out
for lib in damvsnet_amd/ab/libdamvs_base.so "" damvsnet_amd/ab/libdamvs_xshared.so; do
  for dt in f32 bf16; do
    for s in 1 2 3; do
      echo -n "${lib:-product} " >> $out
      DAMVS_LIB=$lib timeout -k 10 120 python -u tools/kbench.py --kernel warp --stage $s --batch 4 --dtype $dt --iters 10 >> $out 2>/dev/null || exit $?
    done
  done
done
cat $out
