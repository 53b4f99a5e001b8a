"""CPU: the oracle (oracle/mvs_oracle.py) against the reference's golden vectors and known answers.

These pin the oracle before it is trusted as the checker of the HIP path.
"""
import numpy as np
import pytest
import torch

from conftest import golden, rel_max
from common import (model_state, forward_inputs, depthnet_inputs, warp_inputs, costreg_input, costreg_state,
                    checksum)
from oracle import mvs_oracle as O

torch.set_num_threads(min(8, torch.get_num_threads()))


def test_fixture_inputs_regenerate():
    """Inputs are regenerated from seeds; the fixture checksums prove they are the ones the reference saw."""
    src, P, hyps = warp_inputs()
    np.testing.assert_allclose(checksum(src, hyps, P), golden("homo_warping")["chk"], rtol=1e-12)
    feats, P, hyps = depthnet_inputs()
    f = np.stack([x.numpy() for x in feats])
    np.testing.assert_allclose(checksum(f, hyps, P), golden("depthnet_cfgA_adaptive")["chk"], rtol=1e-12)
    imgs, proj, dv, _ = forward_inputs(1, 5, 128, 160)
    np.testing.assert_allclose(checksum(imgs, dv, *proj.values()), golden("forward_160x128_48_32_8")["chk"], rtol=1e-12)


@pytest.mark.parametrize("impl", ["grid_sample", "gather"])
def test_homo_warping_golden(impl):
    src, P, hyps = warp_inputs()
    out = O.homo_warping(src, O.compose_proj(P[:, 2]), O.compose_proj(P[:, 0]), hyps, impl=impl)
    assert rel_max(out, golden("homo_warping")["out"]) < 2e-6


def test_identity_warp_known_answer():
    """identity cameras, 6x4 ramp src[c,y,x] = 24c + 6y + x."""
    H, W = 4, 6
    src = torch.arange(2 * H * W, dtype=torch.float32).reshape(1, 2, H, W)
    I = torch.eye(4).unsqueeze(0)
    hyps = torch.full((1, 3, H, W), 500.0)
    for impl in ("grid_sample", "gather"):
        out = O.homo_warping(src, I, I, hyps, impl=impl)[0, 0, 0]
        np.testing.assert_allclose(out[0].numpy(), [0, .35, .95, 1.55, 2.15, 1.25], atol=1e-5)
        np.testing.assert_allclose(out[1].numpy(), [2.5, 5.7, 6.9, 8.1, 9.3, 5.0], atol=1e-5)


@pytest.mark.parametrize("s", [0, 1, 2])
def test_costregnet_golden(s):
    sd = costreg_state(s)
    y = O.costregnet(costreg_input(s), {"cr." + k: v for k, v in sd.items()}, "cr")
    assert rel_max(y, golden("costreg")["logits%d" % s]) < 1e-5


@pytest.mark.parametrize("mode", ["adaptive", "variance"])
def test_depthnet_cfgA_golden(mode):
    g = golden("depthnet_cfgA_" + mode)
    sd = model_state("depthnet_cfgA_" + mode)
    feats, P, hyps = depthnet_inputs()
    out = O.depthnet_stage(2, feats, P, hyps, sd, mode)
    assert rel_max(out["depth"], g["depth"]) < 1e-5
    assert rel_max(out["photometric_confidence"], g["conf"]) < 1e-5
    assert rel_max(out["variance"], g["var"]) < 1e-4
    assert rel_max(out["prob_volume"], g["prob"]) < 1e-5


def test_featurenet_unet_golden():
    """FeatureNet arch_mode="unet" (models/module.py:385-399,430-441; DeConv2dFuse :334-352) vs the reference."""
    from common import featurenet_unet_state
    from damvsnet_amd import synth
    g = golden("featurenet_unet")
    x = torch.from_numpy(synth.images(1, 2, 96, 128, seed=0)[0])
    np.testing.assert_allclose(checksum(x), g["chk"], rtol=1e-12)
    sd = {"feature." + k: v for k, v in featurenet_unet_state().items()}
    with torch.no_grad():
        out = O.feature_net(x, sd, arch_mode="unet")
    for k in ("stage1", "stage2", "stage3"):
        assert rel_max(out[k], g[k]) < 1e-5, k


def test_conditioning_fixture_reproduces():
    """tests/golden/conditioning.npz: the oracle's fp32 cascade at 160x128 against the committed float64
    depths reproduces the committed fp32-vs-fp64 statistics (the e2e GPU gates are multiples of them)."""
    from conftest import pixel_rel
    g = golden("conditioning")
    sd = model_state("forward_160x128_48_32_8")
    imgs, proj, dv, _ = forward_inputs(1, 5, 128, 160)
    with torch.no_grad():
        out = O.cascade_forward(sd, imgs, proj, dv, (48, 32, 8), "adaptive")
    for s in (1, 2, 3):
        pr = pixel_rel(out["stage%d" % s]["depth"].numpy(), g["160x128_48_32_8::s%d_depth64" % s])
        st = np.array([pr.mean(), np.quantile(pr, 0.99), pr.max()])
        np.testing.assert_allclose(st, g["160x128_48_32_8::s%d_stats" % s], rtol=1e-6)


def test_regression_one_hot_known_answer():
    """Softmax/regression KAT: a dominant logit -> depth = that hypothesis, confidence 1, variance 0."""
    D = 8
    hyps = torch.linspace(500, 600, D).view(1, D, 1, 1).repeat(1, 1, 2, 3)
    logits = torch.full((1, D, 2, 3), -1e4)
    logits[:, 5] = 0.0
    out = O.regression(logits, hyps)
    np.testing.assert_allclose(out["depth"].numpy(), hyps[:, 5].numpy(), rtol=1e-6)
    np.testing.assert_allclose(out["photometric_confidence"].numpy(), 1.0, rtol=1e-6)
    np.testing.assert_allclose(out["variance"].numpy(), 0.0, atol=1e-3)


@pytest.mark.parametrize("tag,N,ndepths,mode", [("160x128_48_32_8", 5, (48, 32, 8), "adaptive"),
                                                ("160x128_64_32_8_variance", 3, (64, 32, 8), "variance")])
def test_cascade_forward_golden(tag, N, ndepths, mode):
    g = golden("forward_" + tag)
    sd = model_state("forward_" + tag)
    imgs, proj, dv, _ = forward_inputs(1, N, 128, 160)
    with torch.no_grad():
        out = O.cascade_forward(sd, imgs, proj, dv, ndepths, mode)
    for s in (1, 2, 3):
        o = out["stage%d" % s]
        assert rel_max(o["depth"], g["s%d_depth" % s]) < 1e-5
        assert rel_max(o["photometric_confidence"], g["s%d_conf" % s]) < 1e-5
        assert rel_max(o["variance"], g["s%d_var" % s]) < 1e-4


@pytest.mark.slow
def test_cascade_forward_cfgB_golden():
    g = golden("forward_cfgB_640x512")
    sd = model_state("forward_cfgB_640x512")
    imgs, proj, dv, _ = forward_inputs(1, 5, 512, 640)
    with torch.no_grad():
        out = O.cascade_forward(sd, imgs, proj, dv, (48, 32, 8), "adaptive")
    assert rel_max(out["stage3"]["depth"], g["s3_depth"]) < 1e-5


def test_uncertainty_samples_shapes_and_order():
    """Stage 2/3 hypotheses are ascending per pixel and bracket the previous depth."""
    B, H, W = 1, 16, 24
    cur = torch.full((B, 1, H, W), 700.0)
    var = torch.rand(B, 1, H, W) * 20 + 1
    s = O.uncertainty_aware_samples(cur, var, 8, (B, H, W))
    assert s.shape == (B, 8, H, W)
    assert bool((s[:, 1:] > s[:, :-1]).all())
    assert bool((s[:, 0] <= cur[:, 0] + 1e-3).all()) and bool((s[:, -1] >= cur[:, 0]).all())
