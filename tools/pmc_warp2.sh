#!/usr/bin/env bash
# PMC passes over the warp kernel (kbench, stage $1, B=4); counters listed once to gpurun_out/pmc_avail.txt.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
S=${1:-2}
mkdir -p $R/gpurun_out/pmcw$S
cd /tmp && export TMPDIR=/tmp
[ -s $R/gpurun_out/pmc_avail.txt ] || timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/pmc_avail.txt 2>&1 || true
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
         "SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_VMEM GRBM_GUI_ACTIVE" \
         "TA_BUSY_avr TD_BUSY_avr GRBM_GUI_ACTIVE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
         "TCC_HIT_sum TCC_MISS_sum" "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $R/gpurun_out/pmcw$S/p$i -o run -- python $R/tools/kbench.py --kernel warp --stage $S --batch 4 --iters 3 > $R/gpurun_out/pmcw$S/p$i.log 2>&1 || echo "pass $i failed: $(tail -2 $R/gpurun_out/pmcw$S/p$i.log)"
done
cd $R && python tools/pmc_table.py gpurun_out/pmcw$S | grep -A1 warp_aggregate | head -6
