"""Shared builders for the parity tests (inputs regenerated from the fixture seeds)."""
import json
import os

import numpy as np
import torch

from damvsnet_amd import synth
from damvsnet_amd.weights import synthetic_state_dict, apply_bn_stats

from conftest import GOLDEN, golden, bn_from_golden

SEED = 0


def reference_keys(arch="fpn"):
    with open(os.path.join(GOLDEN, "state_dict_keys.json")) as f:
        return json.load(f)[arch]


def model_state(golden_name=None, arch="fpn", mode=None):
    """Synthetic reference-keyed state_dict, with calibrated BN stats from a fixture.

    ``mode='variance'`` drops DepthNet.weight_net.* (the reference builds it only for 'adaptive').
    """
    if mode is None:
        mode = "variance" if golden_name and "variance" in golden_name else "adaptive"
    tmpl = {k: tuple(v) for k, v in reference_keys(arch).items()
            if mode == "adaptive" or not k.startswith("DepthNet.weight_net.")}
    sd = synthetic_state_dict(tmpl, SEED)
    if golden_name:
        sd = apply_bn_stats(sd, bn_from_golden(golden(golden_name)))
    return sd


def forward_inputs(B, N, H, W):
    proj, ins, dv = synth.cameras(B, N, H, W)
    imgs = synth.images(B, N, H, W, seed=SEED)
    return (torch.from_numpy(imgs), {k: torch.from_numpy(v) for k, v in proj.items()}, torch.from_numpy(dv),
            {k: torch.from_numpy(v) for k, v in ins.items()})


def depthnet_inputs(B=1, N=3, H=256, W=320, D=8, stage_idx=2, C=8):
    scale = 4 // (2 ** stage_idx)
    proj, _, _ = synth.cameras(B, N, H * scale, W * scale)
    P = torch.from_numpy(proj["stage%d" % (stage_idx + 1)])
    f = synth.features(B, N, C, H, W, seed=SEED)
    feats = [torch.from_numpy(np.ascontiguousarray(f[v])) for v in range(N)]
    hyps = torch.from_numpy(synth.stage_hypotheses(B, D, H, W, seed=SEED))
    return feats, P, hyps


def warp_inputs():
    B, C, H, W, D = 1, 4, 12, 16, 5
    proj, _, _ = synth.cameras(B, 3, 4 * H, 4 * W)
    P = torch.from_numpy(proj["stage1"])
    src = torch.from_numpy(np.ascontiguousarray(synth.features(B, 3, C, H, W, seed=SEED)[2]))
    hyps = torch.from_numpy(synth.stage_hypotheses(B, D, H, W, seed=SEED))
    return src, P, hyps


def costreg_input(s):
    C = (32, 16, 8)[s]
    return torch.from_numpy(synth.features(1, 1, C * 8, 16, 24, seed=SEED + 10 + s)[0].reshape(1, C, 8, 16, 24))


def costreg_state(s):
    """CostRegNet-only state_dict (keys without prefix) for fixture ``costreg`` stage s."""
    from damvsnet_amd.layers import CostRegNet
    net = CostRegNet((32, 16, 8)[s], 8)
    sd = synthetic_state_dict(net.state_dict(), SEED + s)
    g = golden("costreg")
    sd = apply_bn_stats(sd, {k.split("::", 2)[2]: g[k] for k in g.files if k.startswith("s%d::bn::" % s)})
    return sd


def featurenet_unet_state():
    """State of a bare FeatureNet(arch_mode="unet") (reference keys without the "feature." prefix, as the
    fixture generator instantiated it) with the calibrated BN stats of tests/golden/featurenet_unet.npz."""
    from damvsnet_amd.frontend import FeatureNet
    net = FeatureNet(base_channels=8, stride=4, num_stage=3, arch_mode="unet")
    sd = synthetic_state_dict(net.state_dict(), SEED)
    return apply_bn_stats(sd, bn_from_golden(golden("featurenet_unet")))


def checksum(*arrs):
    return np.array([float(np.asarray(a, dtype=np.float64).sum()) for a in arrs])
