"""Concurrent-stream diagnosis. Stream A repeats one stage-2 U-Net layer (0..9), the whole
U-Net + prob conv ("unet") or the regression ("regress"); stream B repeats the stage-2 warp; B's volumes are
compared with the warp run alone. With a -DDAMVS_DIAG -DDAMVS_DIAG_WARP_LDS_CAMS=1 build (DAMVS_LIB) the warp
stages its cameras in LDS and records every camera word whose LDS copy differs from global memory (right after
its barrier: kind 1, after the depth walk: kind 2) with the workgroup's HW_ID / LDS_ALLOC / XCC_ID.

    DAMVS_LIB=damvsnet_amd/ab/libdamvs_diaglds.so python tools/diag_streams.py [layers...]
Prints one JSON line per layer."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def take(lib):
    if not hasattr(lib, "damvs_diag_take_warp"):
        return None
    buf = (ctypes.c_uint * (8 + 8 * 64))()
    lib.damvs_diag_take_warp(buf, len(buf))
    n = buf[0]
    recs = []
    for i in range(min(n, 64)):
        r = buf[8 + 8 * i: 16 + 8 * i]
        recs.append({"kind": r[0], "block": r[1], "word": r[2], "seen": "0x%08x" % r[3], "want": "0x%08x" % r[4],
                     "hw_id": "0x%08x" % r[5], "lds_alloc": "0x%08x" % r[6], "xcc": r[7]})
    return {"count": n, "records": recs[:12]}


def main():
    import bench
    from damvsnet_amd.engine import hypotheses, regress, proj_prepare
    from damvsnet_amd import _capi
    lib = _capi.load_library()
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
    warp = lambda: eng.warp_aggregate(feats, None, hyps, rt=rt, layout=_capi.DAMVS_LAYOUT_NHWC)
    with torch.no_grad():
        vol = warp()
        bufs = eng.unet_buffers(2, D, h, w)
        logits = eng.costreg_logits(vol)
        torch.cuda.synchronize()
        ref = vol.clone()
        solo = take(lib)  # records from the solo runs (expected: none)
        print(json.dumps({"layer": "solo", "diag": solo}), flush=True)
        layers = sys.argv[1:] or ["unet", "regress"] + [str(i) for i in range(10)]
        for which in layers:
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
            for trial in range(6):
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
                del outs
            print(json.dumps({"layer": which, "warps_differing": bad, "of": 48, "diag": take(lib)}), flush=True)


if __name__ == "__main__":
    main()
