#!/bin/bash
# Round-5 F (final, no-packed-FP32 warp build): the in-pipeline stage-2 warp counters (bf16, fp32; the bench's
# `traffic` source, refreshed in profiles/r05/ before the bench runs), the full GPU suite, smoke(), the default bench
# line, cfgD / cfgE lines, then the rocprofv3 stats of the default bench command with the roofline-kernel check.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r05F; mkdir -p $O
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return $rc; }
for dt in bf16 f32; do
  sfx=""; [ $dt = f32 ] && sfx="_f32"
  PMC_DTYPE=$dt step timeout -k 10 900 python -u tools/pmc_warp_inpipe.py --out gpurun_out/pmc_inpipe_$dt > $O/pmc_inpipe_$dt.log 2>&1 || { tail -5 $O/pmc_inpipe_$dt.log; exit 1; }
  cp gpurun_out/pmc_inpipe_$dt/pmc_warp_inpipe.json profiles/r05/pmc_warp_inpipe_cfgC_b4$sfx.json && cp profiles/r05/pmc_warp_inpipe_cfgC_b4$sfx.json $O/
  rm -rf gpurun_out/pmc_inpipe_$dt; echo "pmc $dt: $(tail -c 300 $O/pmc_inpipe_$dt.log | tr '\n' ' ')"
done
step timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -8
step timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; echo "smoke rc=$?"; tail -2 $O/smoke.txt
step timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
python -c "import json;d=json.load(open('$O/bench_default.json'));p=d['parity_path'];print('bf16',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['traffic'],'f32',p['value'],p['ms_per_step'],p['roofline']['frac'],'cpu',d['cpu_baseline']['value'])" || tail -5 $O/bench_default.err
for c in cfgD cfgE; do
  step timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err
  python -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c',d['value'],d['ms_per_step'])" || tail -5 $O/bench_$c.err
done
bash tools/gpu_prof.sh; rc=$?
for f in prof_default/run_kernel_stats.csv roofline_check.txt launches.txt steps.txt prof_default.log; do cp gpurun_out/$f $O/$(echo $f | tr / _) 2>/dev/null; done
rm -rf gpurun_out/prof_default gpurun_out/prof_q
exit $rc
