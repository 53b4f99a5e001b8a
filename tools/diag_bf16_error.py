"""Which bf16 rounding drives the bf16 benchmark path's per-pixel depth error?

One DepthNet stage at its cfgC resolution (B=1, 5 views, bf16-representable fp32 features), every variant
against the fp32 HIP path (itself within 4e-5 of the oracle at these sizes, profiles/r02/pytest_gpu_fullsize):
  bf16      the product's bf16 stage (bf16 volume, bf16 folded weights, bf16 activations, fp32 accumulate)
  vol       fp32 engine on the fp32 warp's volume rounded to bf16          (volume storage only)
  weights   fp32 engine with every conv's BN-folded weights rounded to bf16 (weights only)
  vol+wts   both of the above                                               (all but the activations)
Prints per-pixel relative depth error mean / p99 / max per variant and stage as JSON lines.

    python tools/diag_bf16_error.py [stages...]"""
import copy
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def quantise_folded(cr):
    """Copy of a CostRegNet whose BN-folded conv weights (w * gamma / sqrt(var + eps) per output channel) are
    bf16-representable, i.e. what the bf16 engine packs."""
    cr = copy.deepcopy(cr)
    for name in cr.ENCODER + cr.DECODER:
        m = getattr(cr, name)
        bn = m.bn
        scale = (bn.weight / torch.sqrt(bn.running_var + bn.eps)).double()
        w = m.conv.weight.data.double()
        shape = (1, -1, 1, 1, 1) if isinstance(m.conv, torch.nn.ConvTranspose3d) else (-1, 1, 1, 1, 1)
        folded = (w * scale.view(shape)).to(torch.bfloat16).double()
        m.conv.weight.data = (folded / scale.view(shape)).float()
    return cr


def stats(d, r):
    e = np.abs(d.astype(np.float64) - r) / np.abs(r)
    return {"mean": float(e.mean()), "p99": float(np.quantile(e, 0.99)), "max": float(e.max())}


def main():
    from common import model_state, depthnet_inputs
    from damvsnet_amd.cascade import CascadeMVSNet
    from damvsnet_amd.engine import StageEngine, regress
    dev = torch.device("cuda")
    H, W, N, nd = 1184, 1600, 5, (48, 32, 8)
    sd = model_state("depthnet_cfgA_adaptive")
    net = CascadeMVSNet(ndepths=list(nd))
    net.load_state_dict(sd, strict=True)
    net = net.to(dev).eval()
    stages = [int(a) for a in sys.argv[1:]] or [0, 1, 2]
    for s in stages:
        D, C = nd[s], (32, 16, 8)[s]
        h, w = H >> (2 - s), W >> (2 - s)
        feats, P, hyps = depthnet_inputs(B=1, N=N, H=h, W=w, D=D, stage_idx=s, C=C)
        P, hyps = P.to(dev), hyps.to(dev)
        nhwc32 = [f.to(torch.bfloat16).float().permute(0, 2, 3, 1).contiguous().to(dev) for f in feats]
        nhwc16 = [f.to(torch.bfloat16) for f in nhwc32]
        cr, aw = net.cost_regularization[s], net.DepthNet.weight_net[s]
        e32 = StageEngine(cr, aw, "adaptive", torch.float32, dev)
        e16 = StageEngine(cr, aw, "adaptive", torch.bfloat16, dev)
        eq = StageEngine(quantise_folded(cr).to(dev), aw, "adaptive", torch.float32, dev)
        with torch.no_grad():
            ref = e32.forward(nhwc32, P, hyps)[0].cpu().numpy()
            out = {"bf16": e16.forward(nhwc16, P, hyps)[0]}
            vol = e32.warp_aggregate(nhwc32, P, hyps)
            volq = vol.to(torch.bfloat16).float()
            out["vol"] = regress(e32.costreg_logits(volq), hyps)[0]
            out["weights"] = regress(eq.costreg_logits(vol), hyps)[0]
            out["vol+wts"] = regress(eq.costreg_logits(volq), hyps)[0]
            out["split_fp32"] = regress(e32.costreg_logits(vol), hyps)[0]  # the split path itself (control)
        torch.cuda.synchronize()
        line = {"stage": s + 1, "shape": [h, w, D, C]}
        for k, v in out.items():
            line[k] = stats(v.cpu().numpy(), ref)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
