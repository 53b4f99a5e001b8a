#!/bin/bash
# Round-6: the fp32 prob conv + regression in isolation (tools/kbench_prob.py f32), product against the input planes two
# ahead (-DDAMVS_PROB_AHEAD2=1, damvsnet_amd/ab/libdamvs_pahead2.so), the fp32 bench line of both, then the PMC passes.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R && mkdir -p gpurun_out/r06
T=${TAG:-r06q}
timeout -k 10 200 python -u tools/kbench_prob.py 20 f32 > gpurun_out/r06/${T}_kbench_prob_f32.jsonl 2>&1 || exit 3
DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_pahead2.so timeout -k 10 200 python -u tools/kbench_prob.py 20 f32 > gpurun_out/r06/${T}_kbench_prob_f32_ahead2.jsonl 2>&1 || exit 3
grep valu gpurun_out/r06/${T}_kbench_prob_f32.jsonl; echo "== ahead2"; grep valu gpurun_out/r06/${T}_kbench_prob_f32_ahead2.jsonl
TAG=${T} bash tools/gpu_ab.sh "f32|DAMVS_X=1|--dtype f32" "f32 ahead2|DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_pahead2.so|--dtype f32"
bash tools/pmc_cmd.sh r06/${T}_pmc_prob_f32 tools/kbench_prob.py 2 f32 > /dev/null && grep -A2 "prob_regress" gpurun_out/r06/${T}_pmc_prob_f32/table.txt | head -12
