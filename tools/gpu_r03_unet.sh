#!/usr/bin/env bash
# Per-layer U-Net kernel times (kbench --kernel unet, B=4) under rocprofv3 kernel trace, stages 1-3 (default paths)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p $R/gpurun_out/unetl
cd /tmp && export TMPDIR=/tmp
for s in 1 2 3; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d /tmp/unetl/s$s -o run -- python $R/tools/kbench.py --kernel unet --stage $s --batch 4 --iters 3 > $R/gpurun_out/unetl/s$s.log 2>&1 || { tail -3 $R/gpurun_out/unetl/s$s.log; exit 1; }
  echo "== stage $s: $(grep 'per call' $R/gpurun_out/unetl/s$s.log)"
  python - /tmp/unetl/s$s/run_kernel_trace.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "damvs" in r["Kernel_Name"]]
last = rows[-11:]  # one U-Net: 10 convs + the prob conv
for i, r in enumerate(last):
    n = r["Kernel_Name"].replace("damvs::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    print("  %2d %8.1f us  %s" % (i, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, n[:70]))
PY
done
