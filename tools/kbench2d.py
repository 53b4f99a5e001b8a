"""Front-end conv2d microbench (GPU): representative damvs_conv2d layers at cfgC shapes.

  python tools/kbench2d.py [--iters 20] [--dtype bf16|f32] [--only A,B]

Each case is one HipConv2d launch with random weights/inputs; prints us per launch (HIP events on
the launch stream), the MFMA-rate (dense-equivalent TFLOP/s) and the algorithmic HBM rate
(inputs read once + output written once).
"""
import argparse
import os
import sys

import torch
import torch.nn as nn

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

# name: (transposed, k, s, p, op, c0, c1, ngeo, cout, relu, B, Hi, Wi, res_pre, post_up)
CASES = {
    "A conv0.1 8->8 k3 full x5": (False, 3, 1, 1, 0, 8, 0, 0, 8, True, 5, 1184, 1600, False, 0),
    "B inner2 8->32 k1 +up2 x5": (False, 1, 1, 0, 0, 8, 0, 0, 32, False, 5, 1184, 1600, False, 2),
    "B1 inner1 16->32 k1 +up2 x20": (False, 1, 1, 0, 0, 16, 0, 0, 32, False, 20, 592, 800, False, 2),
    "C out3 32->8 k3 full x5": (False, 3, 1, 1, 0, 32, 0, 0, 8, False, 5, 1184, 1600, False, 0),
    "D geo conv2 128+g->128 r4": (False, 3, 1, 1, 0, 128, 0, 1, 128, True, 1, 296, 400, True, 0),
    "E geo conv1 128+g->256 s2": (False, 3, 2, 1, 0, 128, 0, 1, 256, True, 1, 296, 400, False, 0),
    "F deconv 256->128 k5s2 r8": (True, 5, 2, 2, 1, 256, 0, 0, 128, True, 1, 148, 200, False, 1),
    "G deconv 128->32 k5s2 r4": (True, 5, 2, 2, 1, 128, 0, 0, 32, True, 1, 296, 400, False, 1),
    "H geo conv1 32+32+g->64 s2": (False, 3, 2, 1, 0, 32, 32, 1, 64, True, 1, 592, 800, False, 0),
    "I geo conv1 8+g->16 s2 full": (False, 3, 2, 1, 0, 8, 0, 1, 16, True, 1, 1184, 1600, False, 0),
    "J geo conv2 16+g->16 r2": (False, 3, 1, 1, 0, 16, 0, 1, 16, True, 1, 592, 800, True, 0),
    "K geo conv2 64+g->64 r4": (False, 3, 1, 1, 0, 64, 0, 1, 64, True, 1, 296, 400, True, 0),
    "L dec4 128->64 k3 r4": (True, 3, 1, 1, 0, 128, 0, 0, 64, True, 1, 296, 400, False, 0),
    "M dec5 64->32 k5s2 r2": (True, 5, 2, 2, 1, 64, 0, 0, 32, True, 1, 296, 400, False, 1),
    "N geo conv2 128+g->128 r4 B=4": (False, 3, 1, 1, 0, 128, 0, 1, 128, True, 4, 296, 400, True, 0),
    "O geo conv2 32+g->32 r2 B=4": (False, 3, 1, 1, 0, 32, 0, 1, 32, True, 4, 592, 800, True, 0),
    "P dec 32->16 k3 r2 B=4": (False, 3, 1, 1, 0, 32, 0, 0, 16, True, 4, 592, 800, False, 0),
    "Q geo conv2 32+g->16 r2 B=4": (False, 3, 1, 1, 0, 32, 0, 1, 16, True, 4, 592, 800, True, 0),
    "R dec 64->32 k3 r4 B=4": (False, 3, 1, 1, 0, 64, 0, 0, 32, True, 4, 296, 400, False, 0),
    "S fpn top k4s2 32->8 x20": (True, 4, 2, 1, 0, 32, 0, 0, 8, False, 20, 592, 800, False, 0),
    "T geo dec k3s2 16->8 B=4": (True, 3, 2, 1, 1, 16, 0, 0, 8, True, 4, 592, 800, False, 0),
    "U conv0.1 8->8 k3 full x20": (False, 3, 1, 1, 0, 8, 0, 0, 8, True, 20, 1184, 1600, False, 0),
    "V geo dec 8->8 k3 full B=4": (False, 3, 1, 1, 0, 8, 0, 0, 8, True, 4, 1184, 1600, False, 0),
    "W conv0.0 planes g3->8 k3 x20": (False, 3, 1, 1, 0, 0, 0, 3, 8, True, 20, 1184, 1600, False, 0),
    "X rgb init g4->8 k5 B=4": (False, 5, 1, 2, 0, 0, 0, 4, 8, True, 4, 1184, 1600, False, 0),
    "Y depth init g2->8 k5 B=4": (False, 5, 1, 2, 0, 0, 0, 2, 8, True, 4, 1184, 1600, False, 0),
    "G4 deconv 128->32 k5s2 B=4": (True, 5, 2, 2, 1, 128, 0, 0, 32, True, 4, 296, 400, False, 1),
    "M4 dec5 64->32 k5s2 B=4": (True, 5, 2, 2, 1, 64, 0, 0, 32, True, 4, 296, 400, False, 1),
    "Z4 dec 16->8 k5s2 full B=4": (True, 5, 2, 2, 1, 16, 0, 0, 8, True, 4, 592, 800, False, 1),
    "FA feat conv1.0 8->16 k5s2 x20": (False, 5, 2, 2, 0, 8, 0, 0, 16, True, 20, 1184, 1600, False, 0),
    "FB feat conv2.0 16->32 k5s2 x20": (False, 5, 2, 2, 0, 16, 0, 0, 32, True, 20, 592, 800, False, 0),
    "FC feat conv1.1 16->16 k3 x20": (False, 3, 1, 1, 0, 16, 0, 0, 16, True, 20, 592, 800, False, 0),
    "FD feat conv2.1 32->32 k3 x20": (False, 3, 1, 1, 0, 32, 0, 0, 32, True, 20, 296, 400, False, 0),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    from damvsnet_amd import build
    build.build()
    from damvsnet_amd.frontend_hip import HipConv2d
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    tot = 0.0
    for name, (tr, k, s, p, op, c0, c1, ngeo, cout, relu, B, Hi, Wi, pre, up) in CASES.items():
        if args.only and name.split()[0] not in args.only.split(","):
            continue
        cin = c0 + c1 + ngeo
        conv = (nn.ConvTranspose2d(cin, cout, k, stride=s, padding=p, output_padding=op) if tr
                else nn.Conv2d(cin, cout, k, stride=s, padding=p))
        geo_at = tuple(range(c0 + c1, cin))
        at = dict(c0=c0, c0_at=0, c1=c1, c1_at=c0)
        L = HipConv2d(conv, dt, relu, geo_at=geo_at, **at)
        in0 = torch.randn(B, Hi, Wi, c0, device=dev, generator=g).to(dt)
        in1 = torch.randn(B, Hi, Wi, c1, device=dev, generator=g).to(dt) if c1 else None
        gp = torch.rand(B, Hi, Wi, device=dev, generator=g)
        geo = [(gp, Hi * Wi)] * ngeo
        out = L(B, Hi, Wi, in0, in1, geo=geo)
        Ho, Wo = out.shape[1:3]
        res_pre = torch.randn(out.shape, device=dev, generator=g).to(dt) if pre else None
        res_post = torch.randn(B, Ho // up, Wo // up, out.shape[3], device=dev, generator=g).to(dt) if up else None
        kw = dict(geo=geo, res_pre=res_pre, res_post=res_post, post_up=max(up, 1))
        for _ in range(3):
            L(B, Hi, Wi, in0, in1, **kw)
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(args.iters):
            L(B, Hi, Wi, in0, in1, **kw)
        e1.record(st)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.iters
        tot += us
        taps = (k * k) / (s * s) if tr else k * k
        flop = 2.0 * B * Ho * Wo * cout * cin * taps
        es = 2 if dt == torch.bfloat16 else 4
        byt = es * (B * Hi * Wi * (c0 + c1) + out.numel() + (res_pre.numel() if pre else 0) +
                    (res_post.numel() if up else 0)) + 4 * B * Hi * Wi * ngeo
        print("%-30s %8.1f us  %7.1f TFLOP/s  %6.2f TB/s" % (name, us, flop / us * 1e-6, byt / us * 1e-6), flush=True)
    print("total %.1f us" % tot)
    # HBM ceiling for a read + write stream of these sizes: a device copy (torch) of in0's bytes
    for nb in (606 * 2 ** 20, 121 * 2 ** 20):
        x = torch.empty(nb // 2, device=dev, dtype=torch.bfloat16)
        y = torch.empty_like(x)
        for _ in range(3):
            y.copy_(x)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            y.copy_(x)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.iters
        print("copy %4d MiB -> %4d MiB      %8.1f us  %6.2f TB/s (read + write)" % (nb >> 20, nb >> 20, us, 2 * nb / us * 1e-6))


if __name__ == "__main__":
    main()
