cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
for cfg in "X=1" "DAMVS_ZSLIDE_ZC=8" "DAMVS_ZSLIDE_ZC=32" "DAMVS_CONV2D_WANT_TILES=600" "DAMVS_CONV2D_WANT_TILES=1400" "DAMVS_WARP_MINBLK=1024"; do
  env $cfg timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/sw.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "$cfg rc=$rc"; tail -3 gpurun_out/sw.log; exit $rc; }
  echo "$cfg $(tail -1 gpurun_out/sw.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
