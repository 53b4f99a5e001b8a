#!/bin/bash
# Round-5 K: sub-batch phase offset on the two-stream forward (DAMVS_STREAM_OFFSET: sub-batch 2 starts when sub-batch 1
# reaches that phase): the default bench line (bf16 + parity path), interleaved, two runs per setting.
mkdir -p gpurun_out/r05K; O=gpurun_out/r05K
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return $rc; }
for r in 1 2; do for off in none stage1.hypotheses stage2.geofusion stage3.geofusion; do
  v=$off; [ $off = none ] && v=""
  DAMVS_STREAM_OFFSET=$v step timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench_${off}_$r.json 2> $O/bench_${off}_$r.err
  python -c "import json;d=json.load(open('$O/bench_${off}_$r.json'));p=d['parity_path'];print('$off',$r,'bf16',d['value'],d['ms_per_step'],'f32',p['value'],p['ms_per_step'])" || tail -3 $O/bench_${off}_$r.err
done; done
exit 0
