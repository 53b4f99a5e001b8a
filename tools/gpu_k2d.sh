#!/bin/bash
# conv2d microbench (both dtypes) under a time limit
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python tools/kbench2d.py "$@" > gpurun_out/k2d.log 2>&1; rc=$?
cat gpurun_out/k2d.log | grep -v Warning
exit $rc
