#!/bin/bash
# GPU pass: TESTS (pytest files, "" skips; K = a -k expression), then (BENCH=1) the default bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
TAG=${TAG:-r06}
if [ -n "${TESTS-}" ]; then
  kargs=(); [ -n "${K-}" ] && kargs=(-k "$K")
  timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread $TESTS "${kargs[@]}" > gpurun_out/r06/${TAG}_pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|prescale sweep|e2e cfgC" gpurun_out/r06/${TAG}_pytest.log | tail -40
  [ $rc -eq 0 ] || exit $rc
fi
[ "${BENCH-}" = "1" ] || exit 0
# the default bench line (bf16 headline + the fp32 parity_path block)
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r06/${TAG}_bench_default.json 2> gpurun_out/r06/${TAG}_bench_default.err || exit 5
python -c "import json;d=json.loads(open('gpurun_out/r06/${TAG}_bench_default.json').read().strip().splitlines()[-1]);p=d['parity_path'];print('default',d['value'],d['ms_per_step'],'parity',p['value'],{s:{g:round(v['kernels'][g]['ms'],3) for g in v['kernels']} for s,v in p['hot_path_roofline']['per_stage'].items()})"
