"""Isolated timing of the prob conv + regression (damvs_stage_regress) at the bench config's three stages:
MFMA form (default for bf16) against the VALU prob_regress_kernel (DAMVS_PROB_MFMA=0), with and without the
prob-volume write. One JSON line per (stage, kernel, prob).

    python tools/kbench_prob.py [iters] [f32]     (f32: the fp32 parity path's storage)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(iters=20, dt=None):
    import bench
    H, W, N, nd, dtype, _ = bench.CONFIGS["cfgC"]
    if dt == "f32":
        dtype = torch.float32
    dev = torch.device("cuda")
    net, _ = bench.build_model(nd, dtype, dev)
    B = 4
    g = torch.Generator(device=dev).manual_seed(0)
    for s, scale in ((0, 4), (1, 2), (2, 1)):
        D, h, w = nd[s], H // scale, W // scale
        eng = net.DepthNet.engine(s, net.cost_regularization[s], dev)
        c0 = (torch.randn(B, D, h, w, 8, generator=g, device=dev) * 0.5).to(dtype)
        hyps = (500 + torch.rand(B, D, h, w, generator=g, device=dev) * 400).sort(1).values.contiguous()
        scratch = torch.empty(B, D, h, w, device=dev)
        for kern in ("mfma", "valu"):
            os.environ["DAMVS_PROB_MFMA"] = "1" if kern == "mfma" else "0"
            for want_prob in (True, False):
                for _ in range(3):
                    eng.regress_c0(c0, hyps, want_prob=want_prob, scratch=scratch)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(iters):
                    eng.regress_c0(c0, hyps, want_prob=want_prob, scratch=scratch)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / iters
                vox = B * D * h * w
                alg = vox * 8 * c0.element_size() + vox * 4 + (vox * 4 if want_prob else 0) + 3 * B * h * w * 4
                print(json.dumps({"stage": s + 1, "D": D, "hw": [h, w], "B": B, "kernel": kern, "prob_write": want_prob,
                                  "ms": round(ms, 4), "alg_GBps": round(alg / ms / 1e6, 1),
                                  "hbm_frac": round(alg / ms / 1e6 / 8000, 3)}), flush=True)
        os.environ.pop("DAMVS_PROB_MFMA", None)


if __name__ == "__main__":
    main(*(int(a) if a.isdigit() else a for a in sys.argv[1:]))
