#!/usr/bin/env bash
# PMC passes (SQ / GRBM only, one pass per group, kernel trace only) over kbench2d case(s) $1 with
# DAMVS_CONV2D_WIDE=$2; CSVs under gpurun_out/pmcw$2/, summarised by tools/pmc_table.py.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
ONLY=${1:-N}; W=${2:-1}
OUT="$R/gpurun_out/pmcw$W"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_LDS_ADDR_CONFLICT SQ_INST_LEVEL_LDS"; do
  i=$((i+1))
  DAMVS_CONV2D_WIDE=$W timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
    python "$R/tools/kbench2d.py" --iters 2 --only "$ONLY" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
cd "$R" && python tools/pmc_table.py "$OUT" | tee "$OUT/summary.txt"
