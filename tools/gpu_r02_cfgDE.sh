#!/usr/bin/env bash
# cfgD / cfgE bench lines (no CPU baseline) and the one-GPU rehearsal of the depth-sharded cfgD mode (4 ranks as
# threads; a functional run, not a speed figure).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
for c in cfgD cfgE; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1 || { tail -5 gpurun_out/bench_$c.log; exit 1; }
  grep '^{"metric"' gpurun_out/bench_$c.log | tail -1 > gpurun_out/bench_${c}_line.json
  echo "$c: $(python -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["hot_path_roofline"]["per_map"])' gpurun_out/bench_${c}_line.json)"
done
timeout -k 10 400 python -u bench.py --config cfgD --shard depth --emulate 4 --no-cpu-baseline > gpurun_out/bench_cfgD_shard.log 2>&1 || { tail -5 gpurun_out/bench_cfgD_shard.log; exit 1; }
grep '^{"metric"' gpurun_out/bench_cfgD_shard.log | tail -1 > gpurun_out/bench_cfgD_shard_line.json; cut -c1-300 gpurun_out/bench_cfgD_shard_line.json
