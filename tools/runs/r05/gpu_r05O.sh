#!/bin/bash
# Round-5 O: N = 7 unrolled split warp in the product -- the full GPU suite (stream tests with N = 7 cases), smoke, the
# cfgD line and the default line.
mkdir -p gpurun_out/r05O; O=gpurun_out/r05O
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return $rc; }
step timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -8
step timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; echo "smoke rc=$?"
step timeout -k 10 400 python -u bench.py --config cfgD --no-cpu-baseline > $O/bench_cfgD.json 2> $O/bench_cfgD.err
python -c "import json;d=json.load(open('$O/bench_cfgD.json'));print('cfgD',d['value'],d['ms_per_step'],d['parity_path']['value'])" || tail -3 $O/bench_cfgD.err
step timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
python -c "import json;d=json.load(open('$O/bench_default.json'));p=d['parity_path'];print('default bf16',d['value'],d['ms_per_step'],'f32',p['value'],'cpu',d['cpu_baseline']['value'])" || tail -3 $O/bench_default.err
exit 0
