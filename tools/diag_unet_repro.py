"""Diagnose run-to-run differences of the bf16 U-Net (x-pair conv11 on/off via DAMVS_CONV_XPAIR set by
the caller): runs costreg_logits repeatedly on one volume and reports, per run, which regions of
the workspace (the U-Net's level buffers) and the logits differ from run 0.

  DAMVS_CONV_XPAIR=1 python tools/diag_unet_repro.py [--D 64 --stage 0 --runs 6]
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--D", type=int, default=64)
    ap.add_argument("--stage", type=int, default=0)
    ap.add_argument("--runs", type=int, default=6)
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--H", type=int, default=32)
    ap.add_argument("--W", type=int, default=80)
    ap.add_argument("--save", default=None, help="torch.save the --buf snapshots (bf16) here")
    ap.add_argument("--buf", default="c0")
    args = ap.parse_args()
    from common import model_state, depthnet_inputs
    from damvsnet_amd import _capi
    from damvsnet_amd.cascade import CascadeMVSNet
    from damvsnet_amd.engine import StageEngine
    _capi.load_library()
    s, D = args.stage, args.D
    C = (32, 16, 8)[s]
    net = CascadeMVSNet(ndepths=[48, 32, 8])
    net.load_state_dict(model_state("depthnet_cfgA_adaptive"), strict=True)
    feats, P, hyps = depthnet_inputs(B=args.B, N=3, H=args.H, W=args.W, D=D, stage_idx=s, C=C)
    dev = torch.device("cuda")
    eng = StageEngine(net.cost_regularization[s], net.DepthNet.weight_net[s], "adaptive", torch.bfloat16, dev)
    nhwc = [f.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(dev) for f in feats]
    vol = eng.warp_aggregate(nhwc, P.to(dev), hyps.to(dev))
    B, D, h, w, _ = vol.shape
    print("XPAIR env=%s  vol %s" % (os.environ.get("DAMVS_CONV_XPAIR"), tuple(vol.shape)), flush=True)
    snaps = []
    for r in range(args.runs):
        lg = eng.costreg_logits(vol)
        torch.cuda.synchronize()
        ws = eng.workspace(B, 2, D, h, w)
        snaps.append((lg.clone(), ws.clone()))
    al = lambda x: (x + 255) & ~255
    V, es, bb = B * D * h * w, 2, 8
    o = al(B * 1 * 12 * 4)
    if C * es > 16:
        o += 2 * al(B * h * w * C * es)
    names = [("vol", V * C * es)] + [("c%d" % i, z * es) for i, z in enumerate(
        [V * bb, V // 8 * 2 * bb, V // 8 * 2 * bb, V // 64 * 4 * bb, V // 64 * 4 * bb, V // 512 * 8 * bb, V // 512 * 8 * bb])]
    names.append(("logits", V * 4))
    layout = []
    for nm, z in names:
        layout.append((nm, o, o + z))
        o += al(z)
    print("workspace layout:", [(nm, a0, a1) for nm, a0, a1 in layout], flush=True)
    if args.save:
        a0, a1 = [(x, y) for nm, x, y in layout if nm == args.buf][0]
        torch.save([sw[a0:a0 + (a1 - a0) // B].cpu().view(torch.bfloat16) for _, sw in snaps], args.save)  # batch 0
    l0, w0 = snaps[0]
    region = 1 << 16
    for r, (l, wsr) in enumerate(snaps[1:], 1):
        dl = (l != l0)
        a, b = w0.view(torch.uint8), wsr.view(torch.uint8)
        n = a.numel() // region * region
        dw = (a[:n] != b[:n]).view(-1, region).any(1).nonzero().flatten().tolist()
        tail = bool((a[n:] != b[n:]).any())
        print("run %d: logits differ at %d of %d (max |d| %.3g); workspace %d bytes, differing 64 KiB regions %s%s"
              % (r, int(dl.sum()), dl.numel(), float((l - l0).abs().max()), a.numel(),
                 dw[:40], " +tail" if tail else ""), flush=True)
        a8, b8 = w0.view(torch.uint8), wsr.view(torch.uint8)
        for nm, a0, a1 in layout:
            d = (a8[a0:a1] != b8[a0:a1]).nonzero().flatten()
            if d.numel():
                print("   %s: %d bytes differ, first at +%d" % (nm, d.numel(), int(d[0])), flush=True)
        if dl.any():
            idx = dl.nonzero()[:8].tolist()
            print("   first differing logits (b, d, y, x):", idx, flush=True)


if __name__ == "__main__":
    main()
