#!/usr/bin/env bash
# Runtime-view-count warp pipeline: warp / stage / full-size parity (incl. N = 3, 7, 11), then cfgD and cfgE bench
# lines (tree vs HEAD build) and cfgC with the unrolled N = 5 pipeline vs the runtime one (DAMVS_WARP_RUNTIME_VIEWS=1).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_sharded.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_views.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_views.log | tail -8
[ $rc -eq 0 ] || exit $rc
line() { python -c 'import json,sys; d=json.loads(sys.stdin.read()); h=d["hot_path_roofline"]["per_stage"]; print(d["value"], d["ms_per_step"], d["roofline"]["frac"], [round(h[s]["kernels"]["warp"]["ms"], 3) for s in h])'; }
for c in cfgD cfgE; do
  for v in tree base; do
    if [ $v = base ]; then export DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_base.so; else unset DAMVS_LIB; fi
    timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/bench_v.log 2>&1 || { tail -5 gpurun_out/bench_v.log; exit 1; }
    [ $v = tree ] && grep '^{"metric"' gpurun_out/bench_v.log | tail -1 > gpurun_out/bench_${c}_line.json
    echo "$c $v: $(grep '^{"metric"' gpurun_out/bench_v.log | tail -1 | line)"
  done
done
unset DAMVS_LIB
for v in 0 1 0 1; do
  DAMVS_WARP_RUNTIME_VIEWS=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/bench_v.log 2>&1 || { tail -5 gpurun_out/bench_v.log; exit 1; }
  echo "cfgC runtime_views=$v: $(grep '^{"metric"' gpurun_out/bench_v.log | tail -1 | line)"
done
