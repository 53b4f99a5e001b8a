#!/bin/bash
# Round-5 H: same-box A/B of the bf16 wide-conv AG change: the default bench line (no CPU baseline, bf16 + parity path)
# on the product and on the pre-change build (ab/libdamvs_preag.so, commit b69facc), interleaved, three each.
mkdir -p gpurun_out/r05H; O=gpurun_out/r05H
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return $rc; }
for r in 1 2 3; do for v in preag prod; do
  L=damvsnet_amd/libdamvs.so; [ $v = preag ] && L=damvsnet_amd/ab/libdamvs_preag.so
  DAMVS_LIB=$L step timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-parity-path > $O/bench_${v}_$r.json 2> $O/bench_${v}_$r.err
  python -c "import json;d=json.load(open('$O/bench_${v}_$r.json'));print('$v',$r,d['value'],d['ms_per_step'],d['ms_per_stage']['stage3.geofusion'])" || tail -3 $O/bench_${v}_$r.err
done; done
exit 0
