#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06a
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "conv0 or cfgC_e2e or torch_frontend or range_status" > gpurun_out/r06a/pytest_conv0.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r06a/pytest_conv0.log | tail -20
[ $rc -eq 0 ] || exit $rc
for v in "" "0"; do
  DAMVS_CONV0_DZ=$v timeout -k 10 300 python -u tools/unet_layers.py --dtype f32 --only conv0 > gpurun_out/r06a/layers_dz_${v:-def}.txt 2>&1 || exit 3
  echo "== DZ=${v:-default}"; grep conv0 gpurun_out/r06a/layers_dz_${v:-def}.txt
done
for v in "2,1" "4,2" "2,2"; do
  DAMVS_CONV0_DZ=$v timeout -k 10 300 python -u tools/unet_layers.py --dtype f32 --only conv0 --stages 2,3 > gpurun_out/r06a/layers_dz_$v.txt 2>&1; echo "== DZ=$v"; grep conv0 gpurun_out/r06a/layers_dz_$v.txt
done
for v in "" "0"; do
  DAMVS_CONV0_DZ=$v timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --dtype f32 --no-cpu-baseline --no-shard-latency > gpurun_out/r06a/bench_f32_dz_${v:-def}.json 2> gpurun_out/r06a/bench_f32_dz_${v:-def}.err || exit 4
  echo "bench DZ=${v:-def}"; python -c "import json;d=json.loads(open('gpurun_out/r06a/bench_f32_dz_${v:-def}.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])"
done
