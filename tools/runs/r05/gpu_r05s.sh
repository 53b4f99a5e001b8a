#!/bin/bash
# Round-5 s: the even-view-count stage tests (blocked layout), then the cfgE bench line (FeatureNet view groups under
# the 2 GiB operand bound).
mkdir -p gpurun_out/r05s; O=gpurun_out/r05s
timeout -k 10 300 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "even_views or channel_blocked" > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 500 python -u bench.py --config cfgE --no-cpu-baseline > $O/bench_cfgE.json 2> $O/bench_cfgE.err; rc=$?
python -c "import json;d=json.load(open('$O/bench_cfgE.json'));print('cfgE',d['value'],d['ms_per_step'],'f32',d['parity_path']['value'])" || tail -5 $O/bench_cfgE.err
exit $rc
