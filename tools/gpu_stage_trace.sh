R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider -x -k "hypotheses or depthnet or stage" 2>&1 | tail -2 || exit 1
cd /tmp && export TMPDIR=/tmp
for s in 1 2 3; do timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/unet_s$s -o run -- python $R/tools/kbench.py --kernel stage --stage $s --iters 3 > /dev/null 2>&1 || exit 1; done
echo ok
