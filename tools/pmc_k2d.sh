#!/bin/bash
# PMC passes over tools/kbench2d.py cases (one counter group per pass, kernel-trace only), then the per-kernel table.
#   bash tools/pmc_k2d.sh <name> <dtype> <cases>      e.g. bash tools/pmc_k2d.sh k2d_f32 f32 N,E,F
R=${GRAFT_REPO_ROOT:-$(pwd)}
NAME=$1; DT=$2; CASES=$3
OUT=$R/gpurun_out/$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_WAVES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU" \
         "FETCH_SIZE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE" \
         "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
    python $R/tools/kbench2d.py --dtype $DT --only $CASES --iters 3 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
cd $R && python tools/pmc_table.py $OUT > $OUT/table.txt && cat $OUT/table.txt
