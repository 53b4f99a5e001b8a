#!/usr/bin/env bash
# conv2d case N L1-tag PMC (wide vs gather kernel) + in-pipeline A/B of the prob conv (MFMA opt-in vs VALU).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
DAMVS_CONV2D_WIDE=1 bash tools/pmc_deep.sh pmcN_wide $R/tools/kbench2d.py --iters 2 --only N || exit 1
DAMVS_CONV2D_WIDE=0 bash tools/pmc_deep.sh pmcN_gather $R/tools/kbench2d.py --iters 2 --only N || exit 1
cd "$R"
python tools/pmc_table.py gpurun_out/pmcN_wide | grep -A1 "conv2d" | head -4
python tools/pmc_table.py gpurun_out/pmcN_gather | grep -A1 "conv2d" | head -4
for v in ${SKIP_PM:+}; do
  env $v timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_pm.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/bench_pm.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); h=d["hot_path_roofline"]["per_stage"]; print(d["value"], [h[s]["kernels"]["regress"]["ms"] for s in h])')"
done
