#!/bin/bash
# Round-6: fp32 per-step kernel profile, then the bf16 wide-kernel A/B: A two chunks ahead (-DDAMVS_WIDE_APD=2,
# damvsnet_amd/ab/libdamvs_apd2.so) against the product (one ahead).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06m}
TAG=$T bash tools/gpu_prof_f32.sh > /dev/null || exit 3
cd $R
head -30 gpurun_out/${T}_steps_f32.txt | cut -c1-150
for v in prod apd2; do
  if [ $v = prod ]; then L=""; else L=$R/damvsnet_amd/ab/libdamvs_apd2.so; fi
  DAMVS_LIB=$L timeout -k 10 200 python -u tools/kbench2d.py --dtype bf16 > gpurun_out/r06/${T}_k2d_bf16_$v.txt 2>&1 || exit 7
done
paste gpurun_out/r06/${T}_k2d_bf16_prod.txt gpurun_out/r06/${T}_k2d_bf16_apd2.txt | grep " us" | awk -F'\t' '{print $1 " || " $2}' | cut -c1-150
TAG=${T} bash tools/gpu_ab.sh "prod|DAMVS_X=1|--no-parity-path" "apd2|DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_apd2.so|--no-parity-path" "prod2|DAMVS_X=1|--no-parity-path" "apd2b|DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_apd2.so|--no-parity-path"
