#!/bin/bash
# Round-5 G (final, after the bf16 wide-conv AG change): cfgD / cfgE lines and the rocprofv3 stats of the default bench
# command with the roofline-kernel check (the suite and the default line: r05ad).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r05G; mkdir -p $O
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return $rc; }
for c in cfgD cfgE; do
  step timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err
  python -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c',d['value'],d['ms_per_step'])" || tail -5 $O/bench_$c.err
done
bash tools/gpu_prof.sh; rc=$?
for f in prof_default/run_kernel_stats.csv roofline_check.txt launches.txt steps.txt prof_default.log; do cp gpurun_out/$f $O/$(echo $f | tr / _) 2>/dev/null; done
rm -rf gpurun_out/prof_default gpurun_out/prof_q
exit $rc
