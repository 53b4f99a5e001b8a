#!/bin/bash
# Round-5 M (final tree): the full GPU suite and smoke().
mkdir -p gpurun_out/r05M; O=gpurun_out/r05M
step() { "$@"; rc=$?; [ $rc -ge 124 ] && { echo "step failed hard (rc=$rc): $*"; exit $rc; }; return $rc; }
step timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1
grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -8
step timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.txt
exit 0
