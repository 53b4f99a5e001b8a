#!/bin/bash
# Round-5 r (final): the full GPU suite, smoke(), the default bench line (bf16 headline + fp32 parity path + CPU
# baseline), and cfgD / cfgE lines. Stops at the first hard failure.
mkdir -p gpurun_out/r05r; O=gpurun_out/r05r
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return $rc; }
step timeout -k 10 1100 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -8
step timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; echo "smoke rc=$?"; tail -2 $O/smoke.txt
step timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
python -c "import json;d=json.load(open('$O/bench_default.json'));p=d['parity_path'];print('bf16',d['value'],d['ms_per_step'],d['roofline']['frac'],'f32',p['value'],p['ms_per_step'],p['roofline']['frac'],'cpu',d['cpu_baseline'])" || tail -5 $O/bench_default.err
for c in cfgD cfgE; do
  step timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err
  python -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c',d['value'],d['ms_per_step'])" || tail -5 $O/bench_$c.err
done
exit 0
