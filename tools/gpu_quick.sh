R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_gpu_frontend.py -q -p no:cacheprovider > gpurun_out/pytest_fe.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_fe.log | tail -20
[ $rc -le 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r7 -o run -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_bench7.log 2>&1; rc=$?
echo "prof rc=$rc"; tail -1 $R/gpurun_out/prof_bench7.log
exit $rc
