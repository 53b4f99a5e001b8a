R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd $R
for k in "warp 1" "warp 2" "warp 3" "probreg 2" "hyp 2" "unet 2"; do set -- $k; timeout -k 10 120 python tools/kbench.py --kernel $1 --stage $2 --iters 10 2>&1 | grep "per call" || exit 1; done
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "TA_BUSY_avr TD_BUSY_avr GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $R/gpurun_out/pmc/p$i -o run -- python $R/tools/kbench.py --kernel warp --stage 2 --iters 3 > $R/gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc/p$i.log; }
done
echo done
