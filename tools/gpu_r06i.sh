R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/r06/r06i_bench_default.json 2> gpurun_out/r06/r06i_bench_default.err || exit 5
python -c "import json;d=json.loads(open('gpurun_out/r06/r06i_bench_default.json').read().strip().splitlines()[-1]);print('default',d['value'],d['ms_per_step'],'parity',d.get('parity_path',{}).get('value'))"
for dt in f32 bf16; do
  timeout -k 10 300 python -u tools/layer_times.py --dtype $dt --top 80 > gpurun_out/r06/r06i_layers2d_$dt.txt 2>&1 || exit 6
  grep "per group" gpurun_out/r06/r06i_layers2d_$dt.txt
done
timeout -k 10 200 python -u tools/kbench2d.py --dtype f32 > gpurun_out/r06/r06i_k2d_f32.txt 2>&1 || exit 7
timeout -k 10 200 python -u tools/kbench2d.py --dtype bf16 > gpurun_out/r06/r06i_k2d_bf16.txt 2>&1 || exit 7
bash tools/pmc_k2d.sh r06/r06i_pmc_k2d_f32 f32 N,F,E
