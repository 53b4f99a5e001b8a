#!/usr/bin/env bash
# Three-way bench A/B, alternating: the working tree, the HEAD build (damvsnet_amd/ab/libdamvs_base.so,
# tools/build_ab.sh) and the working tree under an environment switch ($1, e.g. DAMVS_WARP_NO_PIPE=1).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
sw=${1:-DAMVS_WARP_NO_PIPE=1}
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    -k "$PYTEST_K" > gpurun_out/pytest_ab3.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_ab3.log | tail -8
  [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  for v in tree base "$sw"; do
    case $v in
      tree) envs="DAMVS_DUMMY=0" ;;
      base) envs="DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_base.so" ;;
      *) envs="$v" ;;
    esac
    env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/bench_ab3.log 2>&1 || { tail -5 gpurun_out/bench_ab3.log; exit 1; }
    echo "$v: $(grep '^{"metric"' gpurun_out/bench_ab3.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); h=d["hot_path_roofline"]["per_stage"]; print(d["value"], d["ms_per_step"], {k: round(v, 3) for k, v in d["ms_per_stage"].items() if v > 0.5}, [[round(h[s]["kernels"][k]["ms"], 3) for k in ("warp", "unet")] for s in h])')"
  done
done
