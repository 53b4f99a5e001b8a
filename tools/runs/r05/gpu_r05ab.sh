#!/bin/bash
# Round-5 ab: stage-3 one-lane warp (C 8) with the unrolled N = 5 view loop (ab/libdamvs_c8unr.so) against the
# runtime loop (product), bf16 B=1 and B=4.
mkdir -p gpurun_out/r05ab; O=gpurun_out/r05ab
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return $rc; }
for b in 1 4; do for v in prod c8unr prod c8unr; do
  L=damvsnet_amd/libdamvs.so; [ $v = c8unr ] && L=damvsnet_amd/ab/libdamvs_c8unr.so
  DAMVS_LIB=$L step timeout -k 10 120 python -u tools/kbench.py --kernel warp --stage 3 --dtype bf16 --batch $b --iters 50 > $O/kb_${v}_b$b.txt 2>&1
  echo "$v b$b: $(tail -1 $O/kb_${v}_b$b.txt)"
done; done
exit 0
