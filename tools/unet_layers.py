"""Per-layer times of the CostRegNet (models/module.py:510-541) at the benchmark shapes (GPU).

  python tools/unet_layers.py [--dtype f32|bf16] [--config cfgC] [--batch 4] [--iters 10] [--stages 1,2,3]

Each layer runs alone through damvs_costreg_layer on synthetic activations (random, finite) and is timed with HIP
events on the launch stream. Per layer: ms, algorithmic FLOPs (27-tap 3D conv / transposed conv, useful MACs only) and
bytes (input + output, + the skip tensor the deconvs add in place), and the fraction of max(FLOPs / MFMA ceiling,
bytes / 8 TB/s) -- the ceiling is the split-f16 one (2.5 / 3 PFLOP/s) for fp32, 2.5 PFLOP/s for bf16.
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402

NAMES = ("conv0", "conv1", "conv2", "conv3", "conv4", "conv5", "conv6", "conv7", "conv9", "conv11")
# (input level, output level, cin multiple of base, cout multiple of base, transposed)
SPEC = ((0, 0, None, 1, False), (0, 1, 1, 2, False), (1, 1, 2, 2, False), (1, 2, 2, 4, False), (2, 2, 4, 4, False),
        (2, 3, 4, 8, False), (3, 3, 8, 8, False), (3, 2, 8, 4, True), (2, 1, 4, 2, True), (1, 0, 2, 1, True))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--config", default="cfgC")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--stages", default="1,2,3")
    ap.add_argument("--only", default="", help="comma-separated layer names (conv0,conv11,...): time only these")
    args = ap.parse_args()
    H, W, N, nd, _, _ = bench.CONFIGS[args.config]
    dtype = torch.float32 if args.dtype == "f32" else torch.bfloat16
    es = 4 if args.dtype == "f32" else 2
    peak = 2.5e15 / 3 if args.dtype == "f32" else 2.5e15
    dev = torch.device("cuda")
    net, _ = bench.build_model(nd, dtype, dev)
    total = 0.0
    g = torch.Generator(device=dev).manual_seed(0)
    for s in (int(x) - 1 for x in args.stages.split(",")):
        scale = (4, 2, 1)[s]
        h, w, D, C = H // scale, W // scale, nd[s], (32, 16, 8)[s]
        eng = net.DepthNet.engine(s, net.cost_regularization[s], dev)
        base = eng.base
        B = args.batch
        vol = (0.1 * torch.randn(B, D, h, w, C, device=dev, generator=g)).to(dtype)
        bufs = [(0.1 * torch.randn(t.shape, device=dev, generator=g)).to(dtype) for t in eng.unet_buffers(B, D, h, w)]
        lv = lambda l: (D >> l) * (h >> l) * (w >> l)  # noqa: E731
        st_total = 0.0
        for li, (lin, lout, cm_in, cm_out, tr) in enumerate(SPEC):
            if args.only and NAMES[li] not in args.only.split(","):
                continue
            src = vol if li == 0 else bufs[(None, 0, 1, 2, 3, 4, 5, 6, 4, 2)[li]]
            dst = bufs[(0, 1, 2, 3, 4, 5, 6, 4, 2, 0)[li]]
            cin = C if cm_in is None else cm_in * base
            cout = cm_out * base
            keep = dst.clone() if tr else None
            with torch.no_grad():
                for _ in range(2):
                    eng.unet_layer(li, D, h, w, src, dst)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    eng.unet_layer(li, D, h, w, src, dst)
                e1.record()
                torch.cuda.synchronize()
                if tr:
                    dst.copy_(keep)  # the deconvs accumulate in place: keep the skip values finite
            ms = e0.elapsed_time(e1) / args.iters
            vout = B * lv(lout)
            flops = 2.0 * vout * cout * cin * 27 / (8 if tr else 1)  # transposed s2: each output sees 1/8 of the taps
            byts = (B * lv(lin) * cin + vout * cout * (2 if tr else 1)) * es
            roof = max(flops / peak, byts / 8e12) * 1e3
            st_total += ms
            print("stage%d %-6s %4d->%-4d %s  %8.3f ms  %7.1f TFLOP/s  %6.0f GB/s  roofline %.3f ms  frac %.2f"
                  % (s + 1, NAMES[li], cin, cout, "T" if tr else " ", ms, flops / ms / 1e9, byts / ms / 1e6, roof,
                     roof / ms), flush=True)
        print("stage%d U-Net total %.3f ms" % (s + 1, st_total), flush=True)
        total += st_total
    print("U-Net total %.3f ms (%s, B=%d)" % (total, args.dtype, args.batch))


if __name__ == "__main__":
    main()
