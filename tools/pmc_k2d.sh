#!/bin/bash
# PMC passes over the conv2d microbench (one pass per counter group; kernel-trace only).
R=${GRAFT_REPO_ROOT:-$(pwd)}
ONLY=${1:-A,B,C}
mkdir -p $R/gpurun_out/pmc2d
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_MFMA" "FETCH_SIZE" "WRITE_SIZE" "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $R/gpurun_out/pmc2d/p$i -o run -- python $R/tools/kbench2d.py --iters 2 --only $ONLY > $R/gpurun_out/pmc2d/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc2d/p$i.log; }
done
echo done
