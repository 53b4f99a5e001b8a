#!/bin/bash
# PMC passes focused on LDS / MFMA / stalls.   bash tools/pmc_lds.sh <outdir> <script> [args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
NAME=$1; shift
OUT=$R/gpurun_out/$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_VALU" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/p$i -o run -- python "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; grep -v "^[WIE]20" $OUT/p$i.log | tail -3; }
done
echo done
