#!/usr/bin/env bash
# Wide conv2d kernel: front-end layer tests, microbench A/B over the env knobs, bench.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_frontend.py -x -q -p no:cacheprovider --timeout 200 \
  --timeout-method thread > gpurun_out/pytest_fe.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_fe.log | tail -8
[ $rc -eq 0 ] || exit $rc
i=0
for v in DAMVS_CONV2D_WIDE=0 DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_base.so DAMVS_CONV2D_WIDE=1; do
  i=$((i+1))
  env $v timeout -k 10 200 python -u tools/kbench2d.py --only D,E,F,K,L,N > gpurun_out/k2d_v$i.log 2>&1; rc=$?
  echo "$v rc=$rc"; grep -E "us|total" gpurun_out/k2d_v$i.log
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_wide.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench_wide.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_stage"])'
exit $rc
