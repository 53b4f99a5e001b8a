#!/bin/bash
# Round-5 x: the warp unit built without packed-FP32 VALU ops (build.py FILE_FLAGS, -fno-slp-vectorize).
# Warp timings against the packed build (ab/libdamvs_pk.so), the wave-level stream diagnosis, the full GPU suite, and
# the default bench line.
mkdir -p gpurun_out/r05x; O=gpurun_out/r05x
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return $rc; }
for s in 1 2 3; do for dt in bf16 f32; do
  for v in pk prod; do
    L=damvsnet_amd/libdamvs.so; [ $v = pk ] && L=damvsnet_amd/ab/libdamvs_pk.so
    DAMVS_LIB=$L step timeout -k 10 120 python -u tools/kbench.py --kernel warp --stage $s --dtype $dt --iters 50 > $O/kb_${v}_s${s}_$dt.txt 2>&1
    echo "$v s$s $dt: $(tail -1 $O/kb_${v}_s${s}_$dt.txt)"
  done
done; done
for dt in f32 bf16; do for st in 0 1; do
  step timeout -k 10 200 python -u tools/diag_warp_streams.py --layout nhwc --layer 1 --dtype $dt --stage $st > $O/diag_${dt}_s$st.jsonl 2>$O/diag_${dt}_s$st.err || { tail -3 $O/diag_${dt}_s$st.err; exit 1; }
  echo "prod $dt stage $st: $(grep -c wave_analysis $O/diag_${dt}_s$st.jsonl) bad launches"
done; done
step timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -8
step timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
python -c "import json;d=json.load(open('$O/bench_default.json'));p=d['parity_path'];print('bf16',d['value'],d['ms_per_step'],d['roofline']['frac'],'f32',p['value'],p['ms_per_step'],p['roofline']['frac'],'cpu',d['cpu_baseline'])" || tail -5 $O/bench_default.err
exit 0
