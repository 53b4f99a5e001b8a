"""Where the fused head (k_head.hip) and the unfused conv11 + prob_mfma disagree, and whether two fused runs agree:
prints the mismatching pixels' (b, y, x) statistics for a few shapes (bf16). GPU diagnostic, not a test."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from common import model_state, depthnet_inputs  # noqa: E402


def run(s, D, B, H, W, dtype=torch.bfloat16):
    from damvsnet_amd.cascade import CascadeMVSNet
    from damvsnet_amd.engine import StageEngine
    C = (32, 16, 8)[s]
    net = CascadeMVSNet(ndepths=[48, 32, 8])
    net.load_state_dict(model_state("depthnet_cfgA_adaptive"), strict=True)
    feats, P, hyps = depthnet_inputs(B=B, N=3, H=H, W=W, D=D, stage_idx=s, C=C)
    eng = StageEngine(net.cost_regularization[s], net.DepthNet.weight_net[s], "adaptive", dtype, torch.device("cuda"))
    nhwc = [f.permute(0, 2, 3, 1).contiguous().to(dtype).cuda() for f in feats]
    out = {}
    for tag, flag in (("f1", "1"), ("f2", "1"), ("u", "0")):
        os.environ["DAMVS_HEAD_FUSE"] = flag
        out[tag] = eng.forward(nhwc, P.cuda(), hyps.cuda())[0].clone()
    torch.cuda.synchronize()
    for a, b in (("f1", "f2"), ("f1", "u")):
        d = (out[a] - out[b]).abs().cpu().numpy()
        bad = np.argwhere(d > 0)
        print("s%d D%d B%d %dx%d %s vs %s: %d / %d pixels differ" % (s, D, B, H, W, a, b, len(bad), d.size), flush=True)
        if len(bad):
            bs, ys, xs = bad[:, 0], bad[:, 1], bad[:, 2]
            print("   b:", np.bincount(bs, minlength=B).tolist(), " y range", ys.min(), ys.max(), " x range", xs.min(),
                  xs.max(), " (y+1)%%8 hist", np.bincount((ys + 1) % 8, minlength=8).tolist(), " (x+1)%%30 hist",
                  np.bincount((xs + 1) % 30, minlength=30).tolist(), flush=True)


if __name__ == "__main__":
    from damvsnet_amd import _capi
    _capi.load_library()
    for case in ((2, 8, 2, 48, 96), (2, 8, 1, 48, 96), (1, 16, 1, 24, 56), (1, 16, 2, 24, 56), (1, 32, 2, 40, 72)):
        run(*case)
