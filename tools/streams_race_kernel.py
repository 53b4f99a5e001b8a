"""Which kernel, running on a concurrent stream, corrupts the stage-2 warp of another stream?
Stream A repeats one stage-2 U-Net layer (RACE_LAYER=0..9), the U-Net + prob conv (RACE_LAYER=unet) or
the regression (RACE_LAYER=regress) while stream B repeats the warp; B's volumes are compared with the
warp run alone."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from damvsnet_amd.engine import hypotheses, regress, block_channels, proj_prepare
    from damvsnet_amd import _capi
    H, W, N, nd, dtype, _ = bench.CONFIGS["cfgC"]
    dev = torch.device("cuda")
    net, _ = bench.build_model(nd, dtype, dev)
    s, C, scale = 1, 16, 2
    h, w, D = H // scale, W // scale, nd[s]
    g = torch.Generator(device=dev).manual_seed(0)
    imgs, proj, dv, _ = bench.make_inputs(2, N, H, W, dev)
    pd = 600 + 100 * torch.rand(2, H // 4, W // 4, device=dev, generator=g)
    pv = 5 + 20 * torch.rand(2, H // 4, W // 4, device=dev, generator=g)
    hyps = hypotheses(dv, D, H, W, scale, pd, pv)
    feats = [torch.randn(2, h, w, C, generator=g, device=dev).to(dtype) for _ in range(N)]
    eng = net.DepthNet.engine(s, net.cost_regularization[s], dev)
    rt = proj_prepare(proj["stage2"])
    fb = block_channels(feats)
    warp = lambda: eng.warp_aggregate(fb, None, hyps, rt=rt, layout=_capi.DAMVS_LAYOUT_CBLOCK)
    vol = warp()
    bufs = eng.unet_buffers(2, D, h, w)
    logits = eng.costreg_logits(vol)
    torch.cuda.synchronize()
    ref = vol.clone()
    which = os.environ.get("RACE_LAYER", "unet")

    def other():
        if which == "unet":
            eng.costreg_logits(vol)
        elif which == "regress":
            regress(logits, hyps)
        else:
            k = int(which)
            src = vol if k == 0 else bufs[(None, 0, 1, 2, 3, 4, 5, 6, 4, 2)[k]]
            eng.unet_layer(k, D, h, w, src, bufs[(0, 1, 2, 3, 4, 5, 6, 4, 2, 0)[k]])

    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    main_s = torch.cuda.current_stream()
    bad = 0
    with torch.no_grad():
        for trial in range(10):
            sa.wait_stream(main_s)
            sb.wait_stream(main_s)
            with torch.cuda.stream(sa):
                for _ in range(8):
                    other()
            outs = []
            with torch.cuda.stream(sb):
                for _ in range(8):
                    outs.append(warp())
            torch.cuda.synchronize()
            bad += sum(not torch.equal(o, ref) for o in outs)
    print("RACE_LAYER=%s: %d of 80 concurrent warps differ" % (which, bad), flush=True)


if __name__ == "__main__":
    main()
