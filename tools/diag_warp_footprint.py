"""Is the in-pipeline warp bound by its L2 working set or by its gather instructions? Times the product warp of
each stage on the pipeline's hypotheses (as bench.warp_roofline) and, with the same instruction stream, with all
source views replaced by view 1 (same feature map and camera: a quarter of the source footprint, identical
addresses per view, identical TA work).

    python tools/diag_warp_footprint.py [iters]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(iters=20):
    import bench
    from damvsnet_amd import _capi
    from damvsnet_amd.engine import hypotheses, proj_prepare, block_channels, warp_blocked
    H, W, N, nd, dtype, _ = bench.CONFIGS["cfgC"]
    dev = torch.device("cuda")
    net, _ = bench.build_model(nd, dtype, dev)
    B = 4
    imgs, proj, dv, _ = bench.make_inputs(B, N, H, W, dev)
    with torch.no_grad():
        feats = net.extract_features(imgs)
        out = net(imgs, proj, dv)
        for stage in (0, 1, 2):
            name = "stage%d" % (stage + 1)
            scale = (4, 2, 1)[stage]
            fs = [f[name].to(dtype).contiguous() for f in feats]
            blocked = warp_blocked(fs[0].shape[-1], fs[0].element_size())
            fb = block_channels(fs) if blocked else fs
            layout = _capi.DAMVS_LAYOUT_CBLOCK if blocked else _capi.DAMVS_LAYOUT_NHWC
            if stage == 0:
                hyps = hypotheses(dv, nd[stage], H, W, scale)
            else:
                prev = out["stage%d" % stage]
                hyps = hypotheses(dv, nd[stage], H, W, scale, prev["depth"], prev["variance"])
            rt = proj_prepare(proj[name])
            eng = net.DepthNet.engine(stage, net.cost_regularization[stage], dev)
            variants = {"product": (fb, rt),
                        "one_source_view": ([fb[0]] + [fb[1]] * (N - 1), rt[:, :1].expand(-1, N - 1, -1).contiguous())}
            for vname, (ff, rr) in variants.items():
                eng.warp_aggregate(ff, None, hyps, rt=rr, layout=layout)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(iters):
                    eng.warp_aggregate(ff, None, hyps, rt=rr, layout=layout)
                e1.record()
                torch.cuda.synchronize()
                print(json.dumps({"stage": stage + 1, "variant": vname, "blocked": blocked,
                                  "ms": round(e0.elapsed_time(e1) / iters, 4)}), flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
