#!/bin/bash
# Round-5 y: with the warp unit free of packed-FP32 ops, the fp32 split warp's unrolled N = 5 view loop
# (ab/libdamvs_f32unr.so; the product takes the runtime loop for fp32) - stream tests, wave-level diagnosis, timings.
mkdir -p gpurun_out/r05y; O=gpurun_out/r05y
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return $rc; }
U=damvsnet_amd/ab/libdamvs_f32unr.so
DAMVS_LIB=$U step timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_streams.py > $O/pytest_streams_f32unr.log 2>&1
echo "f32unr streams: $(tail -1 $O/pytest_streams_f32unr.log)"
for st in 0 1; do
  DAMVS_LIB=$U step timeout -k 10 200 python -u tools/diag_warp_streams.py --layout nhwc --layer 1 --dtype f32 --stage $st > $O/diag_f32unr_s$st.jsonl 2>$O/diag_f32unr_s$st.err || { tail -3 $O/diag_f32unr_s$st.err; exit 1; }
  echo "f32unr stage $st: $(grep -c wave_analysis $O/diag_f32unr_s$st.jsonl) bad launches"
done
for s in 1 2 3; do for v in prod f32unr; do
  L=damvsnet_amd/libdamvs.so; [ $v = f32unr ] && L=$U
  DAMVS_LIB=$L step timeout -k 10 120 python -u tools/kbench.py --kernel warp --stage $s --dtype f32 --iters 50 > $O/kb_${v}_s$s.txt 2>&1
  echo "$v s$s f32: $(tail -1 $O/kb_${v}_s$s.txt)"
done; done
exit 0
