#!/bin/bash
# A/B of the front-end conv2d microbench: HEAD build (damvsnet_amd/ab/libdamvs_base.so) vs working tree.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
echo "== base"; DAMVS_LIB=$R/damvsnet_amd/ab/libdamvs_base.so timeout -k 10 200 python tools/kbench2d.py "$@" || exit $?
echo "== new"; timeout -k 10 200 python tools/kbench2d.py "$@"
