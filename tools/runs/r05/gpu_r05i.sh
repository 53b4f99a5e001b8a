#!/bin/bash
# Round-5 i: conv0 input-plane walk with branch-free interior steps: its parity tests, then conv0 times (fp32, bf16).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "conv0 or costregnet" > gpurun_out/r05i_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r05i_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/unet_layers.py --dtype f32 --only conv0 > gpurun_out/r05i_conv0_f32.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/unet_layers.py --dtype bf16 --only conv0 > gpurun_out/r05i_conv0_bf16.txt 2>&1 || exit $?
grep conv0 gpurun_out/r05i_conv0_*.txt
