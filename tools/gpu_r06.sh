#!/bin/bash
# Round-6 GPU pass: TESTS (pytest files, "" skips; K = a -k expression) then the conv0 layer A/B and the fp32 bench
# A/B (PERF=1).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
TAG=${TAG:-r06}
if [ -n "${TESTS-}" ]; then
  kargs=(); [ -n "${K-}" ] && kargs=(-k "$K")
  timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread $TESTS "${kargs[@]}" > gpurun_out/r06/${TAG}_pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|prescale sweep|e2e cfgC" gpurun_out/r06/${TAG}_pytest.log | tail -40
  [ $rc -eq 0 ] || exit $rc
fi
[ "${PERF-}" = "1" ] || exit 0
for v in "" "0"; do
  DAMVS_CONV0_DZ=$v timeout -k 10 300 python -u tools/unet_layers.py --dtype f32 --only conv0 > gpurun_out/r06/${TAG}_layers_dz_${v:-def}.txt 2>&1 || exit 3
  echo "== DZ=${v:-default}"; grep conv0 gpurun_out/r06/${TAG}_layers_dz_${v:-def}.txt
done
for v in "2,1" "4,2" "2,2"; do
  DAMVS_CONV0_DZ=$v timeout -k 10 300 python -u tools/unet_layers.py --dtype f32 --only conv0 --stages 2,3 > gpurun_out/r06/${TAG}_layers_dz_$v.txt 2>&1; echo "== DZ=$v"; grep conv0 gpurun_out/r06/${TAG}_layers_dz_$v.txt
done
for v in "1" "0"; do
  for dt in f32 bf16; do
    DAMVS_WARP_REUSE=$v timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --dtype $dt --no-cpu-baseline --no-shard-latency > gpurun_out/r06/${TAG}_bench_${dt}_ru$v.json 2> gpurun_out/r06/${TAG}_bench_${dt}_ru$v.err || exit 5
    echo "bench $dt REUSE=$v"; python -c "import json;d=json.loads(open('gpurun_out/r06/${TAG}_bench_${dt}_ru$v.json').read().strip().splitlines()[-1]);hp=d['hot_path_roofline']['per_stage'];print(d['value'],d['ms_per_step'],[round(hp[s]['kernels']['warp']['ms'],3) for s in ('stage1','stage2','stage3')])"
  done
done
for v in "" "0"; do
  DAMVS_CONV0_DZ=$v timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --dtype f32 --no-cpu-baseline --no-shard-latency > gpurun_out/r06/${TAG}_bench_f32_dz_${v:-def}.json 2> gpurun_out/r06/${TAG}_bench_f32_dz_${v:-def}.err || exit 4
  echo "bench f32 DZ=${v:-def}"; python -c "import json;d=json.loads(open('gpurun_out/r06/${TAG}_bench_f32_dz_${v:-def}.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])"
done
