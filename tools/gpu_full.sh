#!/bin/bash
# Full GPU suite, then the default bench line and an fp32 line (each step under its own limit; stops at the first
# failure). Outputs in gpurun_out/r06/<TAG>_*.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
TAG=${TAG:-r06full}
timeout -k 10 900 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r06/${TAG}_pytest_gpu.txt 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR| passed| failed" gpurun_out/r06/${TAG}_pytest_gpu.txt | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r06/${TAG}_bench_default.json 2> gpurun_out/r06/${TAG}_bench_default.err || exit 5
python -c "import json;d=json.loads(open('gpurun_out/r06/${TAG}_bench_default.json').read().strip().splitlines()[-1]);print('default',d['value'],d['ms_per_step'],'parity',d.get('parity_path',{}).get('value'))"
exit $rc
