#!/usr/bin/env bash
# round-3 end: the other benchmark configurations (cfgD: 7 views 64/32/8; cfgE: 11 views 1920x1056) and the
# emulated depth-sharded modes at cfgD (functional rehearsal, 4 ranks as threads on one GPU)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
for c in cfgD cfgE; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -3 gpurun_out/bench_$c.err; exit 1; }
  tail -1 gpurun_out/bench_$c.json | cut -c1-160
done
for m in depth gather; do
  timeout -k 10 300 python -u bench.py --config cfgD --shard $m --emulate 4 --steps 3 --warmup 1 > gpurun_out/bench_shard_$m.json 2> gpurun_out/bench_shard_$m.err || { tail -3 gpurun_out/bench_shard_$m.err; exit 1; }
  tail -1 gpurun_out/bench_shard_$m.json | cut -c1-300
done
