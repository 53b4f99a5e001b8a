"""CPU model of split-bf16 convolution precision against the end-to-end conditioning gates.

Every conv / transposed conv of the oracle forward (oracle/mvs_oracle.py) is replaced by its split-bf16 form:
x = xh + xl (+ xm ...) with bf16 pieces, the products of the chosen piece pairs each exact (a bf16 x bf16 product
fits fp32), summed in float64 and rounded to fp32 once -- the arithmetic of MFMA bf16 instructions accumulating in
fp32, up to the order of the fp32 additions. The per-stage per-pixel relative depth difference against the float64
forward (tests/golden/conditioning.npz) is printed as a multiple of the reference's own fp32-vs-fp64 statistics,
i.e. what tests/test_gpu_parity.py::_check_forward_e2e would measure.

  python tools/split_precision_model.py [--terms 3|6|exact] [--scope unet|all] [--cases 160|all]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from oracle import mvs_oracle as O  # noqa: E402
from common import model_state, forward_inputs  # noqa: E402
from conftest import golden  # noqa: E402

PAIRS = {"h3": [(0, 0), (0, 1), (1, 0)], "h4": [(0, 0), (0, 1), (1, 0), (1, 1)], "2": [(0, 0)], "3": [(0, 0), (0, 1), (1, 0)], "4": [(0, 0), (0, 1), (1, 0), (1, 1)],
         "6": [(0, 0), (0, 1), (1, 0), (0, 2), (2, 0), (1, 1)],
         "h1": [(0, 0)], "h2w": [(0, 0), (0, 1)], "h2x": [(0, 0), (1, 0)]}
F16 = ("h1", "h2w", "h2x", "h3", "h4")  # pieces in f16 (the split-f16 MFMA forms); the others bf16


def pieces(x, n, dt=torch.bfloat16):
    out, r = [], x.double()
    for _ in range(n):
        p = r.float().to(dt).double()
        out.append(p)
        r = r - p
    return out


def make(fn, pairs, xpieces=None):
    def emu(x, w, *a, **k):
        if x.dtype != torch.float32:
            return fn(x, w, *a, **k)
        b = None
        if len(a) >= 1:
            b, a = a[0], a[1:]
        else:
            b = k.pop("bias", None)
        n = 1 + max(max(p) for p in pairs)
        dt = torch.float16 if any(pairs is PAIRS[k] for k in F16) else torch.bfloat16
        xp = pieces(x, n if xpieces is None else xpieces, dt)
        wp = pieces(w, n, dt)
        y = 0
        for i, j in pairs:
            if i < len(xp):
                y = y + fn(xp[i], wp[j], None, *a, **k)
        y = y.float()
        if b is not None:
            shape = [1, -1] + [1] * (y.dim() - 2)
            y = y + b.view(shape)
        return y
    return emu


CASES = [("160x128_48_32_8", "forward_160x128_48_32_8", 128, 160, 5, (48, 32, 8), "adaptive"),
         ("160x128_64_32_8_variance", "forward_160x128_64_32_8_variance", 128, 160, 3, (64, 32, 8), "variance"),
         ("cfgB_640x512", "forward_cfgB_640x512", 512, 640, 5, (48, 32, 8), "adaptive")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--terms", default="3")
    ap.add_argument("--scope", default="all")
    ap.add_argument("--cases", default="160")
    ap.add_argument("--unet", default=None)
    ap.add_argument("--geoff", default=None)
    ap.add_argument("--featurenet", default=None)
    ap.add_argument("--xpieces", type=int, default=None, help="activation pieces (1: activations stored bf16)")
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 8)
    if args.terms != "exact":
        pairs = PAIRS[args.terms]
        if args.scope in ("unet", "all"):
            F.conv3d = make(F.conv3d, pairs, args.xpieces)
            F.conv_transpose3d = make(F.conv_transpose3d, pairs, args.xpieces)
        if args.scope in ("frontend", "all"):
            F.conv2d = make(F.conv2d, pairs, args.xpieces)
            F.conv_transpose2d = make(F.conv_transpose2d, pairs, args.xpieces)
    # per-network overrides: --unet / --geoff / --featurenet <terms>
    if args.unet:
        F.conv3d = make(F.conv3d, PAIRS[args.unet], args.xpieces)
        F.conv_transpose3d = make(F.conv_transpose3d, PAIRS[args.unet], args.xpieces)
    for net, t in (("feature_net", args.featurenet), ("geo_feature_fusion", args.geoff)):
        if not t:
            continue
        orig, c2, t2 = getattr(O, net), F.conv2d, F.conv_transpose2d
        e2, et2 = make(c2, PAIRS[t], args.xpieces), make(t2, PAIRS[t], args.xpieces)

        def wrapped(*a, _o=orig, _e=(e2, et2), _c=(c2, t2), **k):
            F.conv2d, F.conv_transpose2d = _e
            try:
                return _o(*a, **k)
            finally:
                F.conv2d, F.conv_transpose2d = _c
        setattr(O, net, wrapped)
    g = golden("conditioning")
    for case, fixture, H, W, N, nd, mode in CASES:
        if args.cases == "160" and not case.startswith("160"):
            continue
        t0 = time.time()
        sd = model_state(fixture)
        imgs, proj, dv, _ = forward_inputs(1, N, H, W)
        with torch.no_grad():
            out = O.cascade_forward(sd, imgs, proj, dv, nd, mode)
        for s in (1, 2, 3):
            ref = g["%s::s%d_depth64" % (case, s)]
            rm, rp, rx = g["%s::s%d_stats" % (case, s)]
            d = out["stage%d" % s]["depth"].double().numpy()
            pr = np.abs(d - ref) / np.maximum(np.abs(ref), 1e-12)
            m, p, x = pr.mean(), np.quantile(pr, 0.99), pr.max()
            print("terms=%s scope=%s unet=%s geoff=%s fn=%s %-26s stage%d: mean %.2e (%.2fx) p99 %.2e (%.2fx) max %.2e (%.2fx)"
                  % (args.terms, args.scope, args.unet, args.geoff, args.featurenet, case, s, m, m / rm, p, p / rp, x, x / rx), flush=True)
        print("  (%.1f s)" % (time.time() - t0), flush=True)


if __name__ == "__main__":
    main()
