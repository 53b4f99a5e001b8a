#!/bin/bash
# Round-5 check e: the full GPU suite, then the default bench line (bf16 headline + fp32 parity path, no CPU baseline)
# and an fp32 one-stream / two-stream pair. Stops at the first hard failure (exit status >= 124).
mkdir -p gpurun_out
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return 0; }
step timeout -k 10 1100 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r05e_pytest.log 2>&1
grep -E "^FAILED|passed|failed" gpurun_out/r05e_pytest.log | tail -15
step timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05e_bench.json 2> gpurun_out/r05e_bench.err
python -c "import json;d=json.load(open('gpurun_out/r05e_bench.json'));p=d['parity_path'];print('bf16',d['value'],d['ms_per_step'],'f32',p['value'],p['ms_per_step'],p['roofline']['frac'],p['mfma_roofline']['frac'])" || tail -5 gpurun_out/r05e_bench.err
step timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --dtype f32 --streams 1 --no-cpu-baseline > gpurun_out/r05e_bench_f32_s1.json 2> gpurun_out/r05e_bench_f32_s1.err
python -c "import json;d=json.load(open('gpurun_out/r05e_bench_f32_s1.json'));print('f32 1 stream',d['value'],d['ms_per_step'])" || tail -5 gpurun_out/r05e_bench_f32_s1.err
