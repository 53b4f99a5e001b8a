"""BASELINE.json's full-size configs on one GPU: parity and invariants at the benchmark shapes.

Configs (bench.py CONFIGS): cfgC DTU 1600x1184, 5 views, 48/32/8; cfgD DTU 1600x1184, 7 views, 64/32/8 (the
reference's inference default, test_uni.py:77); cfgE Tanks&Temples 1920x1056, 11 views, 64/32/8.

* DepthNet of every stage at its resolution (1/4, 1/2, 1 of the input; C = 32 / 16 / 8), all views, on
  bf16-representable fp32 features (one oracle run serves both paths): the fp32 HIP path against the
  oracle (oracle/mvs_oracle.py, a restatement of models/cas_mvsnet.py:18-134) at the north-star gate,
  per-pixel |depth - ref| / ref <= 1e-3; the bf16 HIP path (the benchmark's kernels) at the stated bf16
  gate, mean <= 5e-4, p99 <= 1e-3 and max <= 5e-3 per-pixel relative depth. (10-40 s of oracle time per case.)
* The bf16 cascade at each config: size-independent properties of the regression
  (models/cas_mvsnet.py:105-124) at every stage -- the depth of each pixel inside its hypothesis
  range, probabilities summing to 1 over D, confidence in [0, 1] -- plus batch independence (two
  copies of one sample give bitwise identical maps) and run-to-run bitwise reproducibility.
"""
import numpy as np
import pytest
import torch

from conftest import pixel_rel
from common import model_state, forward_inputs, depthnet_inputs
from oracle import mvs_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
# name: (H, W, views, ndepths)
CFGS = {"cfgC": (1184, 1600, 5, (48, 32, 8)), "cfgD": (1184, 1600, 7, (64, 32, 8)),
        "cfgE": (1056, 1920, 11, (64, 32, 8))}


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from damvsnet_amd import _capi
    _capi.load_library()


@pytest.mark.parametrize("cfg,s", [(c, s) for c in CFGS for s in (2, 1, 0)])
def test_depthnet_fullres_vs_oracle(cfg, s):
    """One stage at its full-size resolution, all views: fp32 HIP at the 1e-3 per-pixel gate, bf16 HIP at
    the stated bf16 gate, both against one fp32 oracle run on the same (bf16-representable) inputs."""
    from damvsnet_amd.cascade import CascadeMVSNet
    from damvsnet_amd.engine import StageEngine
    H, W, N, nd = CFGS[cfg]
    D, C = nd[s], (32, 16, 8)[s]
    sd = model_state("depthnet_cfgA_adaptive")
    net = CascadeMVSNet(ndepths=list(nd))
    net.load_state_dict(sd, strict=True)
    net = net.to(DEV).eval()
    h, w = H >> (2 - s), W >> (2 - s)
    feats, P, hyps = depthnet_inputs(B=1, N=N, H=h, W=w, D=D, stage_idx=s, C=C)
    feats = [f.to(torch.bfloat16).float() for f in feats]
    with torch.no_grad():
        out = net.DepthNet(s, [f.to(DEV) for f in feats], P.to(DEV), hyps.to(DEV), D, net.cost_regularization[s])
        ref = O.depthnet_stage(s, feats, P, hyps, sd, "adaptive")
        eng = StageEngine(net.cost_regularization[s], net.DepthNet.weight_net[s], "adaptive", torch.bfloat16,
                          torch.device(DEV))
        nhwc = [f.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(DEV) for f in feats]
        d16 = eng.forward(nhwc, P.to(DEV), hyps.to(DEV))[0].cpu().numpy()
    d, r = out["depth"].cpu().numpy(), ref["depth"].numpy()
    assert d.shape == (1, h, w)
    err = pixel_rel(d, r)
    pr = pixel_rel(d16, r)
    print("%s stage%d (%dx%d, D=%d, N=%d): fp32 max %.3e mean %.3e | bf16 mean %.3e p99 %.3e max %.3e"
          % (cfg, s + 1, w, h, D, N, err.max(), err.mean(), pr.mean(), np.quantile(pr, 0.99), pr.max()))
    assert err.max() < 1e-3, (err.max(), err.mean())
    # probabilities: absolute 5e-3 (a fp32 logit difference of a few 1e-3 moves a sharp D = 48 softmax
    # peak by ~1.5e-3; measured max 1.45e-3 at stage 1), the gate stays on depth as north_star states
    assert np.abs(out["prob_volume"].cpu().numpy() - ref["prob_volume"].numpy()).max() < 5e-3
    # bf16 benchmark path (bf16 volume, bf16 BN-folded weights, bf16 U-Net activations, fp32 accumulation and
    # regression): measured max 2.6e-3 / 3.7e-4 / 9.1e-4 (cfgC stages 1-3), p99 <= 5.3e-4, mean <= 7.5e-5 over
    # cfgC/D/E. The three bf16 roundings contribute comparably at stage 1 (tools/diag_bf16_error.py,
    # profiles/r03/diag_bf16_error.jsonl: volume alone max 1.2e-3, weights alone 1.1e-3, both 1.3e-3).
    assert pr.mean() < 5e-4 and np.quantile(pr, 0.99) < 1e-3 and pr.max() < 5e-3, (pr.mean(), pr.max())


@pytest.mark.parametrize("cfg", list(CFGS))
def test_cascade_bf16_fullsize_invariants(cfg):
    from damvsnet_amd.cascade import CascadeMVSNet
    H, W, N, nd = CFGS[cfg]
    net = CascadeMVSNet(ndepths=list(nd), compute_dtype=torch.bfloat16, frontend_dtype=torch.bfloat16)
    net.load_state_dict(model_state("forward_cfgB_640x512"), strict=True)
    net = net.to(DEV).eval()
    imgs, proj, dv, ins = forward_inputs(1, N, H, W)
    rep = lambda t: t.repeat(2, *([1] * (t.dim() - 1))).to(DEV)
    imgs2, proj2, dv2, ins2 = rep(imgs), {k: rep(v) for k, v in proj.items()}, rep(dv), {k: rep(v) for k, v in ins.items()}
    with torch.no_grad():
        o1 = net(imgs2, proj2, dv2, ins2)
        o2 = net(imgs2, proj2, dv2, ins2)
    for s, (h, w, D) in zip(("stage1", "stage2", "stage3"), ((H // 4, W // 4, nd[0]), (H // 2, W // 2, nd[1]), (H, W, nd[2]))):
        st = o1[s]
        depth, prob, hyp, conf = st["depth"], st["prob_volume"], st["depth_values"], st["photometric_confidence"]
        assert depth.shape == (2, h, w) and prob.shape == (2, D, h, w) and hyp.shape == (2, D, h, w)
        assert torch.isfinite(depth).all() and torch.isfinite(prob).all()
        lo, hi = hyp.min(1).values, hyp.max(1).values
        slack = 1e-5 * hi.abs()
        assert bool(((depth >= lo - slack) & (depth <= hi + slack)).all()), s
        assert float((prob.sum(1) - 1).abs().max()) < 1e-4, s
        assert float(conf.min()) >= 0 and float(conf.max()) <= 1 + 1e-5, s
        assert torch.equal(depth[0], depth[1]) and torch.equal(prob[0], prob[1]), s  # batch independence
        assert torch.equal(depth, o2[s]["depth"]) and torch.equal(conf, o2[s]["photometric_confidence"]), s
    assert torch.equal(o1["depth"], o1["stage3"]["depth"])
