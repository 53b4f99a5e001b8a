#!/bin/bash
# Full GPU suite, then the default bench line and an fp32 line (each step under its own limit; stops at the first
# failure; LAYERS=1: then the front end's per-layer times). Outputs in gpurun_out/r06/<TAG>_*.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
TAG=${TAG:-r06full}
timeout -k 10 900 python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r06/${TAG}_pytest_gpu.txt 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR| passed| failed" gpurun_out/r06/${TAG}_pytest_gpu.txt | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r06/${TAG}_bench_default.json 2> gpurun_out/r06/${TAG}_bench_default.err || exit 5
python -c "import json;d=json.loads(open('gpurun_out/r06/${TAG}_bench_default.json').read().strip().splitlines()[-1]);print('default',d['value'],d['ms_per_step'],'parity',d.get('parity_path',{}).get('value'))"
if [ "${LAYERS-}" = "1" ]; then  # per-layer front-end times, both dtypes
  for dt in f32 bf16; do
    timeout -k 10 300 python -u tools/layer_times.py --dtype $dt --top 80 > gpurun_out/r06/${TAG}_layers2d_$dt.txt 2>&1 || exit 6
    grep "per group" gpurun_out/r06/${TAG}_layers2d_$dt.txt
  done
fi
exit $rc
