#!/bin/bash
# Round-5 N: the split warp's view loop unrolled for N = 7 (cfgD; ab/libdamvs_n7.so) against the runtime loop.
mkdir -p gpurun_out/r05N; O=gpurun_out/r05N
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return $rc; }
for dt in bf16 f32; do for s in 1 2 3; do for v in prod n7; do
  L=damvsnet_amd/libdamvs.so; [ $v = n7 ] && L=damvsnet_amd/ab/libdamvs_n7.so
  DAMVS_LIB=$L step timeout -k 10 120 python -u tools/kbench.py --kernel warp --config cfgD --stage $s --dtype $dt --batch 4 --iters 20 > $O/kb_${v}_${dt}_s$s.txt 2>&1
  echo "$v $dt s$s: $(tail -1 $O/kb_${v}_${dt}_s$s.txt)"
done; done; done
exit 0
