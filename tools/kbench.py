"""Kernel microbench at benchmark shapes (GPU): times one hot-path kernel in isolation.

  python tools/kbench.py --kernel warp|unet|probreg|hyp|stage --stage 2 [--config cfgC] [--iters 20]

Inputs are synthetic (random bf16/fp32 features, hypotheses from the real sampling kernel), weights
from bench.build_model. Prints ms per launch (HIP events on the launch stream).
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="warp", choices=["warp", "unet", "probreg", "hyp", "stage"])
    ap.add_argument("--stage", type=int, default=2, help="1..3")
    ap.add_argument("--config", default="cfgC")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--dtype", default=None, choices=["f32", "bf16"], help="default: the config's")
    ap.add_argument("--views", type=int, default=0, help="override the config's view count N")
    ap.add_argument("--layout", default="auto", choices=["auto", "nhwc", "cblock"],
                    help="warp feature layout (auto: the library's choice, damvs_warp_feat_blocked)")
    args = ap.parse_args()
    H, W, N, nd, dtype, _ = bench.CONFIGS[args.config]
    if args.views:
        N = args.views
    if args.dtype:
        dtype = torch.float32 if args.dtype == "f32" else torch.bfloat16
    dev = torch.device("cuda")
    net, _ = bench.build_model(nd, dtype, dev)
    s = args.stage - 1
    scale = (4, 2, 1)[s]
    h, w, D = H // scale, W // scale, nd[s]
    C = (32, 16, 8)[s]
    B = args.batch
    from damvsnet_amd.engine import hypotheses
    imgs, proj, dv, _ = bench.make_inputs(B, N, H, W, dev)
    g = torch.Generator(device=dev).manual_seed(0)
    feats = [torch.randn(B, h, w, C, generator=g, device=dev).to(dtype) for _ in range(N)]
    if s == 0:
        hyps = hypotheses(dv, D, H, W, scale)
    else:
        ps = scale * 2
        pd = 600 + 100 * torch.rand(B, H // ps, W // ps, device=dev, generator=g)
        pv = 5 + 20 * torch.rand(B, H // ps, W // ps, device=dev, generator=g)
        hyps = hypotheses(dv, D, H, W, scale, pd, pv)
    from damvsnet_amd import _capi
    from damvsnet_amd.engine import block_channels, proj_prepare, warp_blocked
    eng = net.DepthNet.engine(s, net.cost_regularization[s], dev)
    P = proj["stage%d" % (s + 1)]
    rt = proj_prepare(P)
    blocked = warp_blocked(C, feats[0].element_size(), N) if args.layout == "auto" else args.layout == "cblock"
    fb = block_channels(feats) if blocked else feats
    layout = _capi.DAMVS_LAYOUT_CBLOCK if blocked else _capi.DAMVS_LAYOUT_NHWC
    vol = eng.warp_aggregate(fb, None, hyps, rt=rt, layout=layout)

    def run():
        if args.kernel == "warp":
            eng.warp_aggregate(fb, None, hyps, rt=rt, layout=layout)
        elif args.kernel == "unet":
            eng.costreg_logits(vol)
        elif args.kernel == "hyp":
            hypotheses(dv, D, H, W, scale, pd, pv)
        else:
            eng.forward(feats, P, hyps)

    with torch.no_grad():
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
    print("%s stage%d %s %s N=%d %s B=%d: %.3f ms per call" % (args.kernel, args.stage, args.config, str(dtype)[6:], N,
                                                         "cblock" if blocked else "nhwc", B,
                                                   e0.elapsed_time(e1) / args.iters))


if __name__ == "__main__":
    main()
