"""Parameter holders for the hot-path layers, with the reference's state_dict keys.

These modules own the weights of the 3D cost-regularisation U-Net and the adaptive
aggregation weight net so that reference checkpoints load with strict=True. They have
no eager compute: the engine (``damvsnet_amd.engine``) folds their BatchNorms and packs
their weights for the HIP kernels once, and re-packs after ``load_state_dict``.

* ``Conv3dBN``            models/module.py:117-159  (Conv3d bias=False + BatchNorm3d + ReLU)
* ``Deconv3dBN``          models/module.py:161-202  (ConvTranspose3d + BatchNorm3d + ReLU)
* ``CostRegNet``          models/module.py:510-541
* ``AggWeightNetVolume``  models/module.py:544-563
"""
from __future__ import annotations

import torch.nn as nn


class _NoEager:
    def forward(self, *a, **k):  # pragma: no cover - guard
        raise RuntimeError("%s has no eager forward; it is executed by the damvsnet_amd HIP engine"
                           % type(self).__name__)


class Conv3dBN(_NoEager, nn.Module):
    def __init__(self, cin, cout, kernel_size=3, stride=1, padding=1):
        super().__init__()
        self.conv = nn.Conv3d(cin, cout, kernel_size, stride=stride, padding=padding, bias=False)
        self.bn = nn.BatchNorm3d(cout, momentum=0.1)
        self.stride, self.kernel_size, self.out_channels = stride, kernel_size, cout


class Deconv3dBN(_NoEager, nn.Module):
    def __init__(self, cin, cout, kernel_size=3, stride=2, padding=1, output_padding=1):
        super().__init__()
        self.conv = nn.ConvTranspose3d(cin, cout, kernel_size, stride=stride, padding=padding,
                                       output_padding=output_padding, bias=False)
        self.bn = nn.BatchNorm3d(cout, momentum=0.1)
        self.stride, self.out_channels = stride, cout


class CostRegNet(_NoEager, nn.Module):
    """3D U-Net: conv0 s1; conv1/3/5 s2 each followed by s1 conv2/4/6; deconvs conv7/9/11 with skips."""

    ENCODER = ("conv0", "conv1", "conv2", "conv3", "conv4", "conv5", "conv6")
    DECODER = ("conv7", "conv9", "conv11")

    def __init__(self, in_channels, base_channels=8):
        super().__init__()
        b = base_channels
        self.in_channels, self.base_channels = in_channels, b
        self.conv0 = Conv3dBN(in_channels, b)
        self.conv1 = Conv3dBN(b, 2 * b, stride=2)
        self.conv2 = Conv3dBN(2 * b, 2 * b)
        self.conv3 = Conv3dBN(2 * b, 4 * b, stride=2)
        self.conv4 = Conv3dBN(4 * b, 4 * b)
        self.conv5 = Conv3dBN(4 * b, 8 * b, stride=2)
        self.conv6 = Conv3dBN(8 * b, 8 * b)
        self.conv7 = Deconv3dBN(8 * b, 4 * b)
        self.conv9 = Deconv3dBN(4 * b, 2 * b)
        self.conv11 = Deconv3dBN(2 * b, b)
        self.prob = nn.Conv3d(b, 1, 3, stride=1, padding=1, bias=False)


class AggWeightNetVolume(_NoEager, nn.Module):
    """Per-voxel visibility weight: ReLU(BN(k2 * ReLU(BN(sum_c k1_c x_c)))). ``conv0`` is unused (:561)."""

    def __init__(self, in_channels=32):
        super().__init__()
        self.in_channels = in_channels
        self.conv0 = Conv3dBN(in_channels, 1, kernel_size=1, padding=0)
        self.w_net = nn.Sequential(Conv3dBN(in_channels, 1, kernel_size=1, padding=0),
                                   Conv3dBN(1, 1, kernel_size=1, padding=0))
