"""Stage-isolated parity diagnostic (GPU): where does the full forward diverge from the oracle?

Runs the oracle forward on CPU capturing per-stage inputs, then feeds each GPU component the
oracle's own inputs: FeatureNet, GeoFeatureFusion (PyTorch-ROCm), hypotheses and DepthNet (HIP).
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from common import model_state, forward_inputs  # noqa: E402
from oracle import mvs_oracle as O  # noqa: E402


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    d = (a - b).abs()
    pr = d / b.abs().clamp_min(1e-12)
    return "max_rel %.3e  pix_rel max %.3e p99 %.3e mean %.3e" % (
        (d.max() / b.abs().max()).item(), pr.max().item(), torch.quantile(pr.flatten()[:1 << 24].float(), 0.99).item(),
        pr.mean().item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="forward_cfgB_640x512")
    ap.add_argument("--H", type=int, default=512)
    ap.add_argument("--W", type=int, default=640)
    ap.add_argument("--deterministic", action="store_true")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    args = ap.parse_args()
    if args.deterministic:
        torch.backends.cudnn.deterministic = True
        torch.backends.cudnn.benchmark = False
    from damvsnet_amd.cascade import CascadeMVSNet
    from damvsnet_amd.engine import hypotheses
    torch.set_num_threads(16)
    sd = model_state(args.tag)
    net = CascadeMVSNet(ndepths=[48, 32, 8], compute_dtype=torch.bfloat16 if args.dtype == "bf16" else torch.float32)
    net.load_state_dict(sd)
    net = net.cuda().eval()
    imgs, proj, dv, ins = forward_inputs(1, 5, args.H, args.W)
    g = np.load(os.path.join(REPO, "tests", "golden", args.tag + ".npz"))
    cu = lambda t: t.cuda()
    N = imgs.shape[1]
    with torch.no_grad():
        feats = [O.feature_net(imgs[:, v], sd) for v in range(N)]
        gfe = net.extract_features(cu(imgs))
        for s in ("stage1", "stage2", "stage3"):
            print("features", s, rel(gfe[1][s], feats[1][s]))
        depth = var = conf = None
        for s in range(3):
            name = "stage%d" % (s + 1)
            fs = [f[name] for f in feats]
            if s >= 1:
                rgb = F.interpolate(imgs[:, 0], scale_factor=1.0 / 2 ** (2 - s), mode="bilinear", align_corners=False)
                dl = F.interpolate(depth.unsqueeze(1), scale_factor=2, mode="bilinear", align_corners=False)
                cl = F.interpolate(conf.unsqueeze(1), scale_factor=2, mode="bilinear", align_corners=False)
                ref0 = O.geo_feature_fusion(rgb, dl, cl, dv, s, fs[0], sd)
                gpu0 = net.GeoFeatureFusionNet(cu(rgb).contiguous(memory_format=torch.channels_last), cu(dl), cu(cl),
                                               cu(dv), s, cu(fs[0]))
                print(name, "geofusion", rel(gpu0, ref0))
                fs[0] = ref0
            hy = O.stage_hypotheses(s, dv, depth, var, net.ndepths[s], args.H, args.W, (4, 2, 1)[s])
            ghy = hypotheses(cu(dv), net.ndepths[s], args.H, args.W, (4, 2, 1)[s],
                             None if depth is None else cu(depth), None if var is None else cu(var))
            print(name, "hypotheses", rel(ghy, hy))
            out = O.depthnet_stage(s, fs, proj[name], hy, sd)
            gout = net.DepthNet(s, [cu(f) for f in fs], cu(proj[name]), cu(hy), net.ndepths[s],
                                net.cost_regularization[s])
            print(name, "depthnet depth", rel(gout["depth"], out["depth"]))
            print(name, "depthnet var  ", rel(gout["variance"], out["variance"]))
            print(name, "oracle vs golden depth", rel(out["depth"], torch.from_numpy(g["s%d_depth" % (s + 1)])))
            depth, var, conf = out["depth"], out["variance"], out["photometric_confidence"]
        full = net(cu(imgs), {k: cu(v) for k, v in proj.items()}, cu(dv), {k: cu(v) for k, v in ins.items()})
        full2 = net(cu(imgs), {k: cu(v) for k, v in proj.items()}, cu(dv), {k: cu(v) for k, v in ins.items()})
        for s in (1, 2, 3):
            print("full forward stage%d depth vs golden" % s, rel(full["stage%d" % s]["depth"],
                                                                 torch.from_numpy(g["s%d_depth" % s])))
        print("run-to-run equal:", torch.equal(full["depth"], full2["depth"]), rel(full2["depth"], full["depth"]))


if __name__ == "__main__":
    main()
