#!/bin/bash
# Round-5 I: the narrow high-resolution GeoFF decoder layers (bf16): times and PMC (tools/pmc_cmd.sh passes).
mkdir -p gpurun_out/r05I; O=gpurun_out/r05I
timeout -k 10 200 python -u tools/kbench2d.py --dtype bf16 --only G4,M4,Z4,T,X,Y,O,P,Q --iters 20 > $O/kb2d_bf16.txt 2>&1 || { tail -5 $O/kb2d_bf16.txt; exit 1; }
cat $O/kb2d_bf16.txt
timeout -k 10 600 bash tools/pmc_cmd.sh r05I/pmc tools/kbench2d.py --dtype bf16 --only G4,M4,Z4,T,X,Y --iters 2 > $O/pmc_table.txt 2>&1; rc=$?
rm -rf gpurun_out/r05I/pmc/p*/ ; tail -60 $O/pmc_table.txt; exit $rc
