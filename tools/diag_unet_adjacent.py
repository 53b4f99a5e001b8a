"""U-Net layers on level buffers carved back to back from one allocation (as the stage workspace lays them out) against
separate allocations, layer by layer on identical inputs; then with NaN-filled guards between the carved buffers. A
layer whose output differs only when the buffers touch reads past its input or writes past its output. GPU
diagnostic, not a test."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from common import model_state, depthnet_inputs  # noqa: E402

SRC = [None, 0, 1, 2, 3, 4, 5, 6, 4, 2]
DST = [0, 1, 2, 3, 4, 5, 6, 4, 2, 0]


def carve(B, D, H, W, dt, guard_bytes):
    chans = [8, 16, 16, 32, 32, 64, 64]
    shapes = [(B, D >> l, H >> l, W >> l, c) for l, c in zip((0, 1, 1, 2, 2, 3, 3), chans)]
    es = torch.tensor([], dtype=dt).element_size()
    sizes = [int(np.prod(s)) * es for s in shapes]
    al = lambda x: (x + 255) // 256 * 256
    total = sum(al(s) + guard_bytes for s in sizes) + guard_bytes
    raw = torch.empty(total, dtype=torch.uint8, device="cuda")
    raw.view(torch.float32)[: total // 4].fill_(float("nan"))
    out, o = [], guard_bytes
    for shp, sz in zip(shapes, sizes):
        out.append(raw[o:o + sz].view(dt).view(shp))
        o += al(sz) + guard_bytes
    return raw, out


def main(s=2, D=8, B=1, H=48, W=96, chained=False):
    from damvsnet_amd import _capi
    from damvsnet_amd.cascade import CascadeMVSNet
    from damvsnet_amd.engine import StageEngine
    _capi.load_library()
    C = (32, 16, 8)[s]
    net = CascadeMVSNet(ndepths=[48, 32, 8])
    net.load_state_dict(model_state("depthnet_cfgA_adaptive"), strict=True)
    feats, P, hyps = depthnet_inputs(B=B, N=3, H=H, W=W, D=D, stage_idx=s, C=C)
    dt = torch.bfloat16
    eng = StageEngine(net.cost_regularization[s], net.DepthNet.weight_net[s], "adaptive", dt, torch.device("cuda"))
    nhwc = [f.permute(0, 2, 3, 1).contiguous().to(dt).cuda() for f in feats]
    vol = eng.warp_aggregate(nhwc, P.cuda(), hyps.cuda())
    sep = eng.unet_buffers(B, D, H, W)
    keep = [carve(B, D, H, W, dt, g) for g in (0, 1 << 20)]
    for layer in range(10):
        # identical inputs: copy the separate path's current input / in-place output into both carved sets
        for _, bufs in keep:
            if chained:
                break
            if layer > 0:
                bufs[SRC[layer]].copy_(sep[SRC[layer]])
            if layer >= 7:
                bufs[DST[layer]].copy_(sep[DST[layer]])
        inp = vol if layer == 0 else sep[SRC[layer]]
        eng.unet_layer(layer, D, H, W, inp, sep[DST[layer]])
        ref = sep[DST[layer]].float().cpu().numpy()
        for (raw, bufs), tag in zip(keep, ("adjacent", "guarded")):
            inp = vol if layer == 0 else bufs[SRC[layer]]
            eng.unet_layer(layer, D, H, W, inp, bufs[DST[layer]])
            got = bufs[DST[layer]].float().cpu().numpy()
            d = np.abs(got - ref).max(-1)
            bad = np.argwhere(~(d == 0))
            print("layer %d %s: %d / %d voxels differ%s" % (layer, tag, len(bad), d.size,
                  (" z %d..%d y %d..%d x %d..%d" % (bad[:, 1].min(), bad[:, 1].max(), bad[:, 2].min(), bad[:, 2].max(),
                                                  bad[:, 3].min(), bad[:, 3].max())) if len(bad) else ""), flush=True)


if __name__ == "__main__":
    print("-- inputs copied from the separate path before every layer")
    main()
    print("-- chained: each carved set runs the whole U-Net on its own outputs")
    main(chained=True)
