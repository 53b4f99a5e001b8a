"""Per-layer times of the HIP 2D front-end (FeatureNet + GeoFeatureFusion) inside a cfgC forward.

Each damvs_conv2d layer call is bracketed by HIP events on the current stream after a warm forward; the
table lists ms per call with the layer's shape (kernel, stride, transposed, cin c0+c1(+geo), cout,
input H x W, B), its algorithmic TFLOP/s and GB/s (tensor inputs + fp32 planes + output; residuals not counted)
and its roofline fraction max(FLOPs / 2.5 PFLOP/s, bytes / 8 TB/s) / time. Synchronous per layer (no overlap): a
profile aid, not the bench number.
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
    ap.add_argument("--dtype", choices=["bf16", "f32"], default=None, help="override the config's dtype (f32: the parity path)")
    args = ap.parse_args()
    import bench
    from damvsnet_amd import frontend_hip as F
    H, W, N, nd, dtype, _ = bench.CONFIGS[args.config]
    if args.dtype:
        dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    es = 2.0 if dtype == torch.bfloat16 else 4.0
    # fp32: every product as three split-f16 MFMAs, so the compute ceiling is a third of the dense f16 rate
    peak = 2.5e15 if dtype == torch.bfloat16 else 2.5e15 / 3
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
    ideal = collections.defaultdict(float)
    flops_g = collections.defaultdict(float)
    for lab, L, B, Hi, Wi, in0, in1, ng, oshape, e0, e1 in rec:
        ms = e0.elapsed_time(e1)
        c0 = in0.shape[-1] if in0 is not None else 0
        c1 = in1.shape[-1] if in1 is not None else 0
        cin = c0 + c1 + ng
        px = B * Hi * Wi if L.transposed else B * oshape[1] * oshape[2]  # a transposed conv scatters k^2 taps per input
        flops = 2.0 * px * cin * L.cout * L.kernel * L.kernel
        byts = es * B * Hi * Wi * (c0 + c1) + 4.0 * B * Hi * Wi * ng + es * B * oshape[1] * oshape[2] * oshape[3]
        t_roof = max(flops / peak, byts / 8e12) * 1e3  # ms
        rows.append((ms, lab, "%s %dx%d->%dx%d B%d cin %d+%d+g%d cout %d" % (L.desc, Hi, Wi, oshape[1], oshape[2], B, c0,
                                                                            c1, ng, L.cout),
                     flops / ms / 1e9, byts / ms / 1e6, t_roof / ms))
        agg[lab] += ms
        ideal[lab] += t_roof
        flops_g[lab] += flops
    print("per group (ms):", {k: round(v, 3) for k, v in agg.items()}, "total %.3f" % sum(agg.values()))
    print("per group roofline ms (max(FLOPs/%.2f PF, bytes/8TB/s) per layer):" % (peak / 1e15), {k: round(v, 3) for k, v in ideal.items()},
          "TFLOP/s:", {k: round(flops_g[k] / agg[k] / 1e9, 1) for k in agg})
    for ms, lab, desc, tf, gb, fr in sorted(rows, reverse=True)[:args.top]:
        print("%8.3f ms  %-14s %-58s %7.1f TFLOP/s %7.0f GB/s  roofline %.2f" % (ms, lab, desc, tf, gb, fr))


if __name__ == "__main__":
    main()
