cd $GRAFT_REPO_ROOT
for v in DAMVS_PROB_MFMA=1 DAMVS_PROB_MFMA=0; do for s in 1 2; do env $v timeout -k 10 120 python tools/kbench.py --kernel probreg --stage $s --batch 4 --iters 20 2>&1 | grep "per call" | sed "s/^/$v /" || exit 1; done; done
