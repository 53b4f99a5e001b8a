"""BASELINE.json's full size (DTU 1600x1184, 5 views): parity and invariants at the benchmark shape.

* DepthNet of every stage at its cfgC resolution (stage 3: 1184 x 1600, 8 hypotheses, C = 8; stage
  2: 592 x 800, 32, C = 16; stage 1: 296 x 400, 48, C = 32; ref + 4 sources, fp32): the HIP path against
  the oracle (oracle/mvs_oracle.py, a restatement of models/cas_mvsnet.py:18-134)
  on identical inputs, gated at the north-star tolerance: per-pixel |depth - ref| / ref <= 1e-3.
  (About 10 s of oracle time per stage on the host.)
* The bf16 stage path at the same sizes against the fp32 oracle on bf16-rounded features, at the
  stated bf16 gate (mean <= 5e-3, p99 <= 2e-2 per-pixel relative depth).
* The bf16 cascade at cfgC (48/32/8): size-independent properties of the regression
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
H, W = 1184, 1600


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from damvsnet_amd import _capi
    _capi.load_library()


@pytest.mark.parametrize("s,D,C", [(2, 8, 8), (1, 32, 16), (0, 48, 32)])
def test_depthnet_fullres_vs_oracle(s, D, C):
    """Each stage at its cfgC resolution (1/4, 1/2, 1 of 1184 x 1600), fp32, ref + 4 sources."""
    from damvsnet_amd.cascade import CascadeMVSNet
    sd = model_state("depthnet_cfgA_adaptive")
    net = CascadeMVSNet(ndepths=[48, 32, 8])
    net.load_state_dict(sd, strict=True)
    net = net.to(DEV).eval()
    h, w = H >> (2 - s), W >> (2 - s)
    feats, P, hyps = depthnet_inputs(B=1, N=5, H=h, W=w, D=D, stage_idx=s, C=C)
    with torch.no_grad():
        out = net.DepthNet(s, [f.to(DEV) for f in feats], P.to(DEV), hyps.to(DEV), D, net.cost_regularization[s])
        ref = O.depthnet_stage(s, feats, P, hyps, sd, "adaptive")
    d, r = out["depth"].cpu().numpy(), ref["depth"].numpy()
    assert d.shape == (1, h, w)
    err = pixel_rel(d, r)
    assert err.max() < 1e-3, (err.max(), err.mean())
    # probabilities: absolute 5e-3 (a fp32 logit difference of a few 1e-3 moves a sharp D = 48 softmax
    # peak by ~1.5e-3; measured max 1.45e-3 at stage 1), the gate stays on depth as north_star states
    assert np.abs(out["prob_volume"].cpu().numpy() - ref["prob_volume"].numpy()).max() < 5e-3


@pytest.mark.parametrize("s,D,C", [(2, 8, 8), (1, 32, 16), (0, 48, 32)])
def test_depthnet_bf16_fullres_stated_gate(s, D, C):
    """The benchmark's bf16 stage path (z-streamed conv0 / conv11, banded-MFMA prob conv for D >= 32)
    at each stage's cfgC resolution against the fp32 oracle on the same bf16-rounded features:
    the stated bf16 gate of test_gpu_parity.py, mean <= 5e-3 and p99 <= 2e-2 per-pixel relative depth."""
    from damvsnet_amd.cascade import CascadeMVSNet
    from damvsnet_amd.engine import StageEngine
    sd = model_state("depthnet_cfgA_adaptive")
    net = CascadeMVSNet(ndepths=[48, 32, 8])
    net.load_state_dict(sd, strict=True)
    h, w = H >> (2 - s), W >> (2 - s)
    feats, P, hyps = depthnet_inputs(B=1, N=5, H=h, W=w, D=D, stage_idx=s, C=C)
    feats = [f.to(torch.bfloat16).float() for f in feats]
    eng = StageEngine(net.cost_regularization[s], net.DepthNet.weight_net[s], "adaptive", torch.bfloat16,
                      torch.device(DEV))
    nhwc = [f.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(DEV) for f in feats]
    with torch.no_grad():
        depth = eng.forward(nhwc, P.to(DEV), hyps.to(DEV))[0]
        ref = O.depthnet_stage(s, feats, P, hyps, sd, "adaptive")["depth"].numpy()
    pr = pixel_rel(depth.cpu().numpy(), ref)
    print("bf16 full-size stage%d: mean %.3e p99 %.3e max %.3e" % (s + 1, pr.mean(), np.quantile(pr, 0.99), pr.max()))
    assert pr.mean() < 5e-3 and np.quantile(pr, 0.99) < 2e-2


def test_cascade_bf16_cfgC_invariants():
    from damvsnet_amd.cascade import CascadeMVSNet
    net = CascadeMVSNet(ndepths=[48, 32, 8], compute_dtype=torch.bfloat16, frontend_dtype=torch.bfloat16)
    net.load_state_dict(model_state("forward_cfgB_640x512"), strict=True)
    net = net.to(DEV).eval()
    imgs, proj, dv, ins = forward_inputs(1, 5, H, W)
    rep = lambda t: t.repeat(2, *([1] * (t.dim() - 1))).to(DEV)
    imgs2, proj2, dv2, ins2 = rep(imgs), {k: rep(v) for k, v in proj.items()}, rep(dv), {k: rep(v) for k, v in ins.items()}
    with torch.no_grad():
        o1 = net(imgs2, proj2, dv2, ins2)
        o2 = net(imgs2, proj2, dv2, ins2)
    for s, (h, w, D) in zip(("stage1", "stage2", "stage3"), ((H // 4, W // 4, 48), (H // 2, W // 2, 32), (H, W, 8))):
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
