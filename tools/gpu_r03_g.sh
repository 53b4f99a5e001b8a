#!/usr/bin/env bash
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" && mkdir -p gpurun_out
DAMVS_LIB=damvsnet_amd/ab/libdamvs_diaglds.so timeout -k 10 300 python -u tools/diag_streams2.py 0 > gpurun_out/diag2_lds_rays.log 2>&1 && echo "rays done" &&
DAMVS_LIB=damvsnet_amd/ab/libdamvs_diaglds32.so timeout -k 10 300 python -u tools/diag_streams2.py 0 7 > gpurun_out/diag2_lds32.log 2>&1 && echo "b32 done"
for f in gpurun_out/diag2_lds_rays.log gpurun_out/diag2_lds32.log; do echo "== $f"; python3 - "$f" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if not line.startswith('{'): continue
    d = json.loads(line)
    print(d['layer'], 'differ', d['differ_kernel_compare'], 'of', d['outputs'], 'diag_records', d.get('diag_records'))
    for r in d.get('diag_first', []):
        print('   kind', r[0], 'block', r[1], 'lane', r[2] >> 8, 'view*8+comp', r[2] & 255, 'seen %08x want %08x' % (r[3], r[4]), 'hw_id %08x' % r[5])
    for x in d['details'][:3]:
        print('   ', {k: x.get(k) for k in ('pixels_differ', 'lane_group_hist')})
PY
done
