#!/bin/bash
# Round-5 z: in-pipeline counters of the stage-3 warp (bf16 one-lane C 8 kernel) and the stage-1 split warp (C 32),
# on the no-packed-FP32 build.
mkdir -p gpurun_out/r05z; O=gpurun_out/r05z
export TMPDIR=/tmp
PMC_WARP_KERNEL="warp_aggregate_kernel<unsigned short, 8" PMC_WARP_GRID=0 timeout -k 10 500 python -u tools/pmc_warp_inpipe.py --out $O/s3 --passes 0,1,2,3,4 > $O/s3.txt 2>&1 || { tail -5 $O/s3.txt; exit 1; }
PMC_WARP_KERNEL="warp_split_kernel<unsigned short, 32" PMC_WARP_GRID=0 timeout -k 10 300 python -u tools/pmc_warp_inpipe.py --out $O/s1 --passes 0,1,2,3 > $O/s1.txt 2>&1 || { tail -5 $O/s1.txt; exit 1; }
PMC_WARP_GRID=0 timeout -k 10 300 python -u tools/pmc_warp_inpipe.py --out $O/s2 --passes 0,1 > $O/s2.txt 2>&1 || { tail -5 $O/s2.txt; exit 1; }
rm -rf $O/s1/p* $O/s2/p* $O/s3/p*
for s in s1 s2 s3; do echo "== $s"; python -c "import json;d=json.load(open('$O/$s/pmc_warp_inpipe.json'));print(json.dumps(d['summary'].get('pipeline')))"; done
