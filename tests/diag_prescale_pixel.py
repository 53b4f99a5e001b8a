"""The worst pixel of the fp32 prescale sweep (tests/test_gpu_parity.py test_fp32_prescale_feature_scale_sweep): HIP vs
the float64 oracle's probability volume there (top planes), to tell a near-tie flip from a precision loss.

  python tools/diag_prescale_pixel.py [--case 0] [--scale 100]"""
import argparse
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
from common import model_state, depthnet_inputs  # noqa: E402
from oracle import mvs_oracle as O  # noqa: E402

CASES = [(0, 128, 160, 48, 5), (1, 256, 320, 32, 5), (2, 512, 640, 8, 5), (1, 592, 800, 32, 5)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", type=int, default=0)
    ap.add_argument("--scale", type=float, default=100.0)
    a = ap.parse_args()
    from damvsnet_amd.cascade import CascadeMVSNet
    s, h, w, D, N = CASES[a.case]
    C = (32, 16, 8)[s]
    sd = model_state("depthnet_cfgA_adaptive")
    net = CascadeMVSNet(ndepths=[48, 32, 8])
    net.load_state_dict(sd, strict=True)
    net = net.cuda().eval()
    feats, P, hyps = depthnet_inputs(B=1, N=N, H=h, W=w, D=D, stage_idx=s, C=C)
    feats = [f * a.scale for f in feats]
    sd64 = {k: (v.double() if torch.is_floating_point(v) else v) for k, v in sd.items()}
    with torch.no_grad():
        out = net.DepthNet(s, [f.cuda() for f in feats], P.cuda(), hyps.cuda(), D, net.cost_regularization[s])
        r32 = O.depthnet_stage(s, feats, P, hyps, sd, "adaptive")
        r64 = O.depthnet_stage(s, [f.double() for f in feats], P.double(), hyps.double(), sd64, "adaptive")
        vol64 = O.aggregate([f.double() for f in feats], P.double(), hyps.double(), sd64, s, "adaptive", "grid_sample")
        lg64 = O.costregnet(vol64, sd64, "cost_regularization.%d" % s)
        vol32 = O.aggregate(feats, P, hyps, sd, s, "adaptive", "grid_sample")
        lg32 = O.costregnet(vol32, sd, "cost_regularization.%d" % s)
    d = out["depth"].cpu().double().numpy()
    e = np.abs(d - r64["depth"].numpy()) / r64["depth"].numpy()
    print("HIP vs fp64: max %.3e at %s; pixels >= 1e-3: %d of %d" % (e.max(), np.unravel_index(e.argmax(), e.shape),
                                                                   (e >= 1e-3).sum(), e.size))
    for idx in zip(*np.nonzero(e >= 1e-4)):
        b, y, x = idx
        ph = out["prob_volume"][b, :, y, x].cpu().double().numpy()
        p64 = r64["prob_volume"][b, :, y, x].numpy()
        p32 = r32["prob_volume"][b, :, y, x].double().numpy()
        l64 = lg64.reshape(lg64.shape[0], -1, h, w)[b, :, y, x].numpy()
        l32 = lg32.reshape(lg32.shape[0], -1, h, w)[b, :, y, x].double().numpy()
        top = np.argsort(-p64)[:3]
        print("pixel", idx, "err %.3e" % e[idx], "depth hip %.4f fp32 %.4f fp64 %.4f" % (d[idx], r32["depth"][idx],
                                                                                          r64["depth"][idx]))
        print("  top planes (fp64)", top, "p64", np.round(p64[top], 4), "p32", np.round(p32[top], 4), "hip",
              np.round(ph[top], 4))
        print("  logits fp64", np.round(l64[top], 4), "fp32", np.round(l32[top], 4), "|logit| max %.3g" % np.abs(l64).max())


if __name__ == "__main__":
    main()
