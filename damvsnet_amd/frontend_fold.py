"""Inference copies of the 2D front-end with every BatchNorm folded into its conv / deconv.

``fold_frontend(module, dtype)`` deep-copies FeatureNet or GeoFeatureFusion, folds each eval-mode
BatchNorm2d into the preceding Conv2d / ConvTranspose2d (weight scale + bias), replaces the BN with
identity, and casts the copy to ``dtype`` in channels-last memory. Removes ~100 BN launches per
forward and, for bf16, every autocast cast kernel (the copy's weights are bf16 already). The
originals (and their state_dict) are untouched.
"""
from __future__ import annotations

import copy

import torch
import torch.nn as nn

from .frontend import ConvBNReLU2d, DeconvBNReLU2d, GeoBlock


def _bn_affine(bn):
    inv = torch.rsqrt(bn.running_var.double() + bn.eps)
    scale = bn.weight.double() * inv
    shift = bn.bias.double() - bn.running_mean.double() * scale
    return scale, shift


@torch.no_grad()
def _fold(conv, bn):
    scale, shift = _bn_affine(bn)
    w = conv.weight.double()
    if isinstance(conv, nn.ConvTranspose2d):  # weight [Cin, Cout, k, k]
        w = w * scale.view(1, -1, 1, 1)
    else:  # [Cout, Cin, k, k]
        w = w * scale.view(-1, 1, 1, 1)
    b = shift if conv.bias is None else conv.bias.double() * scale + shift
    conv.weight.copy_(w.to(conv.weight.dtype))
    conv.bias = nn.Parameter(b.to(conv.weight.dtype))


@torch.no_grad()
def fold_frontend(module: nn.Module, dtype=torch.float32) -> nn.Module:
    m = copy.deepcopy(module).eval()
    for sub in list(m.modules()):
        if isinstance(sub, (ConvBNReLU2d, DeconvBNReLU2d)):
            _fold(sub.conv, sub.bn)
            sub.bn = nn.Identity()
        elif isinstance(sub, GeoBlock):
            _fold(sub.conv1, sub.bn1)
            sub.bn1 = nn.Identity()
            _fold(sub.conv2, sub.bn2)
            sub.bn2 = nn.Identity()
            if sub.downsample is not None:
                _fold(sub.downsample[0], sub.downsample[1])
                sub.downsample[1] = nn.Identity()
        elif isinstance(sub, nn.Sequential) and len(sub) >= 2 and isinstance(sub[0], (nn.Conv2d, nn.ConvTranspose2d)) \
                and isinstance(sub[1], nn.BatchNorm2d):
            _fold(sub[0], sub[1])
            sub[1] = nn.Identity()
    for p in m.parameters():
        p.requires_grad_(False)
    return m.to(dtype=dtype, memory_format=torch.channels_last)
