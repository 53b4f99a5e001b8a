"""Stage-level race bisection: the stage-2 DepthNet pieces (warp, U-Net + prob conv logits, regression,
whole stage forward) for two sub-batches on concurrent streams against the same calls one after another."""
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
    imgs, proj, dv, _ = bench.make_inputs(4, N, H, W, dev)
    pd = 600 + 100 * torch.rand(4, H // 4, W // 4, device=dev, generator=g)
    pv = 5 + 20 * torch.rand(4, H // 4, W // 4, device=dev, generator=g)
    hyps = hypotheses(dv, D, H, W, scale, pd, pv)
    feats = [torch.randn(4, h, w, C, generator=g, device=dev).to(dtype) for _ in range(N)]
    eng = net.DepthNet.engine(s, net.cost_regularization[s], dev)
    P = proj["stage2"]
    parts = [([f[i * 2:(i + 1) * 2] for f in feats], P[i * 2:(i + 1) * 2], hyps[i * 2:(i + 1) * 2]) for i in range(2)]

    only_warp = os.environ.get("RACE_ONLY_WARP") == "1"

    def pieces(fe, pr, hy):
        rt = proj_prepare(pr)
        fb = block_channels(fe)
        if only_warp:
            return {"vol%d" % r: eng.warp_aggregate(fb, None, hy, rt=rt, layout=_capi.DAMVS_LAYOUT_CBLOCK)
                    for r in range(6)}
        vol = eng.warp_aggregate(fb, None, hy, rt=rt, layout=_capi.DAMVS_LAYOUT_CBLOCK)
        logits = eng.costreg_logits(vol)
        dep = regress(logits, hy)[0]
        full = eng.forward(fe, pr, hy)[0]
        return {"vol": vol, "logits": logits, "regress": dep, "stage_forward": full}

    main_s = torch.cuda.current_stream()
    with torch.no_grad():
        seq = [pieces(*p) for p in parts]
        torch.cuda.synchronize()
        for trial in range(8):
            streams = [torch.cuda.Stream() for _ in range(2)]
            outs = []
            for st, p in zip(streams, parts):
                st.wait_stream(main_s)
                with torch.cuda.stream(st):
                    outs.append(pieces(*p))
            torch.cuda.synchronize()
            for i in range(2):
                bad = [k for k in outs[i] if not torch.equal(outs[i][k], seq[i][k])]
                print("trial %d chunk %d: differing %s" % (trial, i, bad or "none"), flush=True)


if __name__ == "__main__":
    main()
