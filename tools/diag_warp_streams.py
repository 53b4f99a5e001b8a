"""Where the stage-2 warp's volume differs when it runs beside U-Net layers on another stream.

  python tools/diag_warp_streams.py [--layout cblock|nhwc] [--layer 0]

Prints, for solo repeats and for runs beside the layer: the number of differing voxels, the batch elements, planes,
rows and lane positions (pixel index mod 64 within the warp's pixel blocks) they fall on, and the largest difference.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="cblock", choices=["cblock", "nhwc"])
    ap.add_argument("--layer", type=int, default=0)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--stage", type=int, default=1, choices=[0, 1])
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    from common import model_state
    from test_gpu_streams import _perturb
    from damvsnet_amd.cascade import CascadeMVSNet
    from damvsnet_amd.engine import hypotheses, block_channels, proj_prepare
    from damvsnet_amd import _capi, synth
    DEV = "cuda"
    net = CascadeMVSNet(ndepths=[48, 32, 8], compute_dtype=dt)
    net.load_state_dict(model_state("depthnet_cfgA_adaptive"), strict=True)
    net = net.to(DEV).eval()
    B, N, H, W, s = 2, 5, 1184, 1600, a.stage
    C, D, scale = (32, 48, 4) if s == 0 else (16, 32, 2)
    h, w = H // scale, W // scale
    proj, _, dv = synth.cameras(B, N, H, W)
    P = _perturb(torch.from_numpy(proj["stage%d" % (s + 1)])).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(0)
    pd = 600 + 100 * torch.rand(B, H // 4, W // 4, device=DEV, generator=g)
    pv = 5 + 20 * torch.rand(B, H // 4, W // 4, device=DEV, generator=g)
    hyps = hypotheses(torch.from_numpy(dv).to(DEV), D, H, W, scale, pd, pv) if s else \
        hypotheses(torch.from_numpy(dv).to(DEV), D, H, W, scale)
    feats = [torch.randn(B, h, w, C, generator=g, device=DEV).to(dt) for _ in range(N)]
    eng = net.DepthNet.engine(s, net.cost_regularization[s], torch.device(DEV))

    def report(tag, outs, ref):
        for i, o in enumerate(outs):
            d = (o.float() - ref.float()).abs()
            bad = (d > 0).any(-1)  # [B][D][h][w]
            nb = int(bad.sum())
            rec = {"case": tag, "rep": i, "voxels": nb}
            if nb:
                idx = bad.nonzero()
                rec["batch"] = sorted(set(idx[:, 0].tolist()))
                rec["planes"] = sorted(set(idx[:, 1].tolist()))[:12]
                rec["rows"] = [int(idx[:, 2].min()), int(idx[:, 2].max())]
                rec["cols"] = [int(idx[:, 3].min()), int(idx[:, 3].max())]
                rec["col_mod_32_hist"] = torch.bincount(idx[:, 3] % 32, minlength=32).tolist()
                rec["row_mod_8_hist"] = torch.bincount(idx[:, 2] % 8, minlength=8).tolist()
                rec["maxdiff"] = float(d.max())
                rec["nan"] = int(torch.isnan(o.float()).sum())
            print(json.dumps(rec), flush=True)

    with torch.no_grad():
        rt = proj_prepare(P)
        if a.layout == "cblock":
            fb = block_channels(feats)
            warp = lambda: eng.warp_aggregate(fb, None, hyps, rt=rt, layout=_capi.DAMVS_LAYOUT_CBLOCK)
        else:
            warp = lambda: eng.warp_aggregate(feats, None, hyps, rt=rt)
        vol = warp()
        bufs = eng.unet_buffers(B, D, h, w)
        torch.cuda.synchronize()
        ref = vol.clone()
        report("solo", [warp() for _ in range(a.reps)], ref)
        torch.cuda.synchronize()
        sa, sb, main = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.current_stream()
        layer = a.layer
        src = vol if layer == 0 else bufs[(None, 0, 1, 2, 3, 4, 5, 6, 4, 2)[layer]]
        dst = bufs[(0, 1, 2, 3, 4, 5, 6, 4, 2, 0)[layer]]
        for it in range(2):
            sa.wait_stream(main)
            sb.wait_stream(main)
            with torch.cuda.stream(sa):
                for _ in range(a.reps):
                    eng.unet_layer(layer, D, h, w, src, dst)
            with torch.cuda.stream(sb):
                outs = [warp() for _ in range(a.reps)]
            torch.cuda.synchronize()
            report("beside layer %d (iteration %d)" % (layer, it), outs, ref)
        # same stream, interleaved (no concurrency)
        outs = []
        for _ in range(a.reps):
            eng.unet_layer(layer, D, h, w, src, dst)
            outs.append(warp())
        torch.cuda.synchronize()
        report("interleaved on one stream", outs, ref)


if __name__ == "__main__":
    main()
