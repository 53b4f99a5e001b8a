#!/bin/bash
# Round-6 checkpoint A: the full GPU suite, then the default bench line with its CPU baseline, cfgD and cfgE lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06fa}
timeout -k 10 900 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r06/${T}_pytest_gpu.txt 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR| passed| failed" gpurun_out/r06/${T}_pytest_gpu.txt | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/r06/${T}_bench_default.json 2> gpurun_out/r06/${T}_bench_default.err || exit 5
python -c "import json;d=json.loads(open('gpurun_out/r06/${T}_bench_default.json').read().strip().splitlines()[-1]);print('default',d['value'],d['ms_per_step'],'parity',d['parity_path']['value'],'cpu',d['cpu_baseline'])"
for c in cfgD cfgE; do
  timeout -k 10 600 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/r06/${T}_bench_$c.json 2> gpurun_out/r06/${T}_bench_$c.err || exit 6
  python -c "import json;d=json.loads(open('gpurun_out/r06/${T}_bench_$c.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['ms_per_step'],'parity',d['parity_path']['value'])"
done
