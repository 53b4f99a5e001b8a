#!/bin/bash
# Round-5 ad: bf16 wide conv2d on the AG loop (A fragments from L1 / L2) in the product -- the full GPU suite (stream
# tests included: the ISA pins), smoke, and the default bench line twice.
mkdir -p gpurun_out/r05ad; O=gpurun_out/r05ad
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return $rc; }
step timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -8
step timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; echo "smoke rc=$?"
for r in 1 2; do
  step timeout -k 10 600 python -u bench.py $([ $r = 2 ] && echo --no-cpu-baseline) > $O/bench_default_$r.json 2> $O/bench_default_$r.err
  python -c "import json;d=json.load(open('$O/bench_default_$r.json'));p=d['parity_path'];print('bf16',d['value'],d['ms_per_step'],d['ms_per_stage']['stage3.geofusion'],'f32',p['value'],p['ms_per_step'])" || tail -5 $O/bench_default_$r.err
done
exit 0
