#!/bin/bash
# PMC passes (one counter group per pass, kernel-trace only; the groups of tools/pmc_k2d.sh) over any python command,
# then the per-kernel table (tools/pmc_table.py).   bash tools/pmc_cmd.sh <name> <python args...>
#   e.g. bash tools/pmc_cmd.sh conv0_f32 tools/unet_layers.py --dtype f32 --stages 2 --only conv0 --iters 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
NAME=$1; shift
OUT=$R/gpurun_out/$NAME
mkdir -p $OUT
ARGS=()
for a in "$@"; do [[ $a == tools/* ]] && ARGS+=("$R/$a") || ARGS+=("$a"); done
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_WAVES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU" \
         "FETCH_SIZE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE" \
         "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
    python "${ARGS[@]}" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
cd $R && python tools/pmc_table.py $OUT > $OUT/table.txt && cat $OUT/table.txt
