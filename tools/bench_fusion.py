"""Depth-fusion throughput: reference views fused per second at DTU's final
resolution (1184 x 1600 depth maps, 10 source views as in DTU's pair.txt), GPU kernel
(damvs_fusion_view, HIP events on its stream) vs the oracle's numpy restatement of filter/dypcd.py on
the host (one reference view, single process as the reference's per-scene worker).

  python tools/bench_fusion.py [--H 1184 --W 1600 --nsrc 10 --iters 20 --no-cpu]

Algorithmic bytes per reference view: 4 B x H x W x (1 ref depth + 3 confidences + nsrc source depths
(each read once; the 4-tap lookups hit L2) + 4 depth_avg + 1 mask + 12 xyz).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--H", type=int, default=1184)
    ap.add_argument("--W", type=int, default=1600)
    ap.add_argument("--nsrc", type=int, default=10)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    from test_fusion import plane_scene
    from damvsnet_amd.fusion import fuse_view
    depths, K, E, confs, img = plane_scene(args.nsrc + 1, H=args.H, W=args.W, seed=0)
    cu = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    srcs = [(cu(depths[i]), K[i], E[i]) for i in range(1, args.nsrc + 1)]
    ref, cf = cu(depths[0]), [cu(c) for c in confs]
    for _ in range(3):
        fuse_view(ref, K[0], E[0], srcs, cf)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        fuse_view(ref, K[0], E[0], srcs, cf)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    px = args.H * args.W
    alg = 4 * px * (1 + 3 + args.nsrc + 1) + px + 12 * px
    out = {"metric": "fused reference views/s", "value": round(1e3 / ms, 2), "ms_per_view": round(ms, 4),
           "shape": [args.H, args.W], "nsrc": args.nsrc, "achieved_GBps": round(alg / ms / 1e6, 1),
           "algorithmic_bytes": alg}
    if not args.no_cpu:
        from oracle import fusion_oracle as FO
        t0 = time.perf_counter()
        FO.fuse_view(depths[0], K[0], E[0], [(depths[i], K[i], E[i]) for i in range(1, args.nsrc + 1)], confs,
                     (0.1, 0.15, 0.9), img=img)
        cpu = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(1.0 / cpu, 4), "unit": "views/s", "cores": 1, "kind": "port",
                               "sample": "1 reference view, numpy restatement of filter/dypcd.py"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
