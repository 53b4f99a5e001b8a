#!/bin/bash
# Round-5 check: stream / frontend / range-status tests, wide-kernel kbench (rolling K loop vs AG), per-layer fp32
# front-end times with and without the 32-K gather form, fp32 bench line.
# Stops at the first step that ends in a fault / abort / time limit (exit status >= 124).
mkdir -p gpurun_out
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return 0; }
step timeout -k 10 700 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_frontend.py \
  "tests/test_gpu_parity.py::test_depthnet_range_status" "tests/test_gpu_parity.py::test_cascade_range_status_fp32" \
  > gpurun_out/r05b_pytest.log 2>&1
tail -3 gpurun_out/r05b_pytest.log
# the warp beside conv0 on another stream: the default build and the clamp build (-DDAMVS_WARP_CLAMP, damvsnet_amd/ab)
for dt in f32 bf16; do for st in 1 0; do
  step timeout -k 10 120 python -u tools/diag_warp_streams.py --layout nhwc --dtype $dt --stage $st > gpurun_out/r05b_diag_${dt}_s$st.jsonl 2>&1
  [ -f damvsnet_amd/ab/libdamvs_clamp.so ] && DAMVS_LIB=damvsnet_amd/ab/libdamvs_clamp.so step timeout -k 10 120 python -u tools/diag_warp_streams.py --layout nhwc --dtype $dt --stage $st > gpurun_out/r05b_diag_${dt}_s${st}_clamp.jsonl 2>&1
done; done
grep -c '"voxels": 0' gpurun_out/r05b_diag_*.jsonl
step timeout -k 10 200 python -u tools/kbench2d.py --dtype f32 --only D,E,F,G,L,M,N,O,Q > gpurun_out/r05b_k2d_f32.txt 2>&1
tail -9 gpurun_out/r05b_k2d_f32.txt
DAMVS_WIDE_RS=0 DAMVS_HALO_RS=0 step timeout -k 10 200 python -u tools/kbench2d.py --dtype f32 --only D,F,G,L,M,N,O,Q > gpurun_out/r05b_k2d_f32_ag.txt 2>&1
tail -6 gpurun_out/r05b_k2d_f32_ag.txt
step timeout -k 10 240 python -u tools/layer_times.py --dtype f32 --top 70 > gpurun_out/r05b_layers_f32.txt 2>&1
head -3 gpurun_out/r05b_layers_f32.txt
DAMVS_CONV2D_G32=0 DAMVS_WIDE_RS=0 DAMVS_HALO_RS=0 step timeout -k 10 240 python -u tools/layer_times.py --dtype f32 --top 70 > gpurun_out/r05b_layers_f32_base.txt 2>&1
head -3 gpurun_out/r05b_layers_f32_base.txt
step timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --dtype f32 --no-cpu-baseline > gpurun_out/r05b_bench_f32.json 2> gpurun_out/r05b_bench_f32.err
python -c "import json;d=json.load(open('gpurun_out/r05b_bench_f32.json'));print(d['value'],d['ms_per_step'],d['ms_per_stage'])" || tail -5 gpurun_out/r05b_bench_f32.err
