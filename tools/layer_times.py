"""Per-layer times of the HIP 2D front-end (FeatureNet + GeoFeatureFusion) inside a cfgC forward.

Each damvs_conv2d layer call is bracketed by HIP events on the current stream after a warm forward; the
table lists ms per call with the layer's shape (kernel, stride, transposed, cin c0+c1(+geo), cout,
input H x W, B). Synchronous per layer (no overlap): a profile aid, not the bench number.
  python tools/layer_times.py [--config cfgC] [--batch 4] [--top 40]
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfgC")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    import bench
    from damvsnet_amd import frontend_hip as F
    H, W, N, nd, dtype, _ = bench.CONFIGS[args.config]
    dev = torch.device("cuda")
    net, _ = bench.build_model(nd, dtype, dev)
    imgs, proj, dv, _ = bench.make_inputs(args.batch, N, H, W, dev)
    rec = []
    label = ["features"]
    orig_call = F.HipConv2d.__call__

    def timed(self, B, Hi, Wi, in0=None, in1=None, geo=(), **k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = orig_call(self, B, Hi, Wi, in0, in1, geo, **k)
        e1.record()
        rec.append((label[0], self, B, Hi, Wi, in0, in1, len(geo), out.shape, e0, e1))
        return out

    orig_geo = F.HipGeoFeatureFusion.__call__

    def geo_call(self, *a, **k):
        label[0] = "geofusion s%d" % (a[4] + 1 if len(a) > 4 else k["stage_idx"] + 1)
        try:
            return orig_geo(self, *a, **k)
        finally:
            label[0] = "other"

    with torch.no_grad():
        net(imgs, proj, dv)
        torch.cuda.synchronize()
        F.HipConv2d.__call__ = timed
        F.HipGeoFeatureFusion.__call__ = geo_call
        label[0] = "features"
        net(imgs, proj, dv)
        torch.cuda.synchronize()
    rows = []
    agg = collections.defaultdict(float)
    for lab, L, B, Hi, Wi, in0, in1, ng, oshape, e0, e1 in rec:
        ms = e0.elapsed_time(e1)
        c0 = in0.shape[-1] if in0 is not None else 0
        c1 = in1.shape[-1] if in1 is not None else 0
        rows.append((ms, lab, "%s %dx%d->%dx%d B%d cin %d+%d+g%d cout %d" % (L.desc, Hi, Wi, oshape[1], oshape[2], B, c0,
                                                                            c1, ng, L.cout)))
        agg[lab] += ms
    print("per group (ms):", {k: round(v, 3) for k, v in agg.items()}, "total %.3f" % sum(agg.values()))
    for ms, lab, desc in sorted(rows, reverse=True)[:args.top]:
        print("%8.3f ms  %-14s %s" % (ms, lab, desc))


if __name__ == "__main__":
    main()
