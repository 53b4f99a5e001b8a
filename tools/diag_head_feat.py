"""Fused head: its conv11 + skip feature (diagnostic build, -DDAMVS_DIAG, damvs_head_diag_set) against the unfused
conv11 output (layer by layer through damvs_costreg_layer), twice, on a failing shape. GPU diagnostic, not a test.
  DAMVS_LIB=damvsnet_amd/ab/libdamvs_diag.so python tools/diag_head_feat.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from common import model_state, depthnet_inputs  # noqa: E402


def main(s=2, D=8, B=1, H=48, W=96):
    from damvsnet_amd import _capi
    from damvsnet_amd.cascade import CascadeMVSNet
    from damvsnet_amd.engine import StageEngine
    lib = _capi.load_library()
    lib.damvs_head_diag_set.argtypes = [ctypes.c_void_p]
    C = (32, 16, 8)[s]
    net = CascadeMVSNet(ndepths=[48, 32, 8])
    net.load_state_dict(model_state("depthnet_cfgA_adaptive"), strict=True)
    feats, P, hyps = depthnet_inputs(B=B, N=3, H=H, W=W, D=D, stage_idx=s, C=C)
    dt = torch.bfloat16
    eng = StageEngine(net.cost_regularization[s], net.DepthNet.weight_net[s], "adaptive", dt, torch.device("cuda"))
    nhwc = [f.permute(0, 2, 3, 1).contiguous().to(dt).cuda() for f in feats]
    P, hyps = P.cuda(), hyps.cuda()
    vol = eng.warp_aggregate(nhwc, P, hyps)
    bufs = eng.unet_buffers(B, D, H, W)
    src = [vol, 0, 1, 2, 3, 4, 5, 6, 4, 2]
    dst = [0, 1, 2, 3, 4, 5, 6, 4, 2, 0]
    saved = {}
    for layer in range(10):
        inp = vol if layer == 0 else bufs[src[layer]]
        eng.unet_layer(layer, D, H, W, inp, bufs[dst[layer]])
        saved[layer] = bufs[dst[layer]].float().cpu().numpy()  # every layer's output as written
    ref = bufs[0].float().cpu().numpy()  # conv0 + conv11, bf16
    os.environ["DAMVS_HEAD_FUSE"] = "1"
    feats_f = []
    for _ in range(2):
        dg = torch.zeros(B, D, H, W, 8, device="cuda")
        lib.damvs_head_diag_set(dg.data_ptr())
        eng.forward(nhwc, P, hyps)
        torch.cuda.synchronize()
        lib.damvs_head_diag_set(None)
        feats_f.append(dg.to(dt).float().cpu().numpy())
    for i, f in enumerate(feats_f):
        d = np.abs(f - ref).max(-1)
        bad = np.argwhere(d > 0)
        print("run %d: feature vs unfused conv11: %d / %d voxels differ, max %.3g" % (i, len(bad), d.size, d.max()))
        if len(bad):
            print("   d:", np.bincount(bad[:, 1], minlength=D).tolist(), " y", bad[:, 2].min(), bad[:, 2].max(), " x",
                  bad[:, 3].min(), bad[:, 3].max())
            print("   first:", bad[:5].tolist())
    print("run 0 vs run 1: %d voxels differ" % int((np.abs(feats_f[0] - feats_f[1]).max(-1) > 0).sum()))
    # the forward's workspace after the fused forward: c0 (conv0 output, the skip) and c2 (conv9 output, the input)
    al = lambda x: (x + 255) // 256 * 256
    V, es, N = B * D * H * W, 2, 3
    o = al(B * (N - 1) * 12 * 4) + al(V * C * es)  # rt, vol (8-channel / 16-byte pixels are not blocked)
    sz = [V * 8, V // 8 * 16, V // 8 * 16]
    offs = []
    for i in range(3):
        offs.append(o)
        o += al(sz[i] * es)
    ws = eng.workspace(B, N, D, H, W)

    def check(tag):
        c0 = ws[offs[0]:offs[0] + sz[0] * 2].view(dt).float().cpu().numpy().reshape(B, D, H, W, 8)
        c2 = ws[offs[2]:offs[2] + sz[2] * 2].view(dt).float().cpu().numpy().reshape(B, D // 2, H // 2, W // 2, 16)
        for name, got, want in (("c0", c0, saved[0] if tag == "fused" else ref), ("c2 (conv9 out)", c2, saved[8])):
            d = np.abs(got - want).max(-1)
            bad = np.argwhere(d > 0)
            print("%s forward: workspace %s vs layer path: %d / %d differ" % (tag, name, len(bad), d.size),
                  ("x %d..%d y %d..%d" % (bad[:, 3].min(), bad[:, 3].max(), bad[:, 2].min(), bad[:, 2].max()))
                  if len(bad) else "", flush=True)

    check("fused")
    os.environ["DAMVS_HEAD_FUSE"] = "0"
    eng.forward(nhwc, P, hyps)
    torch.cuda.synchronize()
    check("unfused")
    os.environ["DAMVS_HEAD_FUSE"] = "1"
    # the U-Net alone on the forward's own volume (damvs_costreg_logits: all ten layers, then the prob conv)
    eng.costreg_logits(vol)
    torch.cuda.synchronize()
    check("costreg_logits")
    # every level of the workspace after costreg_logits against the layer that wrote it last
    Ls = [(0, 9, 8, 0), (1, 1, 16, 1), (2, 8, 16, 1), (3, 3, 32, 2), (4, 7, 32, 2), (5, 5, 64, 3), (6, 6, 64, 3)]
    szs = [V * 8, V // 8 * 16, V // 8 * 16, V // 64 * 32, V // 64 * 32, V // 512 * 64, V // 512 * 64]
    o = al(B * (N - 1) * 12 * 4) + al(V * C * es)
    for ci, li, ch, lev in Ls:
        off = o + sum(al(szs[j] * es) for j in range(ci))
        got = ws[off:off + szs[ci] * 2].view(dt).float().cpu().numpy().reshape(B, D >> lev, H >> lev, W >> lev, ch)
        d = np.abs(got - saved[li]).max(-1)
        bad = np.argwhere(d > 0)
        print("c%d (layer %d out, level %d): %d / %d differ" % (ci, li, lev, len(bad), d.size),
              ("z %d..%d y %d..%d x %d..%d" % (bad[:, 1].min(), bad[:, 1].max(), bad[:, 2].min(), bad[:, 2].max(),
                                             bad[:, 3].min(), bad[:, 3].max())) if len(bad) else "", flush=True)


if __name__ == "__main__":
    main()
