"""2D front-end of the cascade: feature pyramid and geometry-aware reference-feature fusion.

These produce the hot path's inputs. The modules here own the parameters
and the reference's state_dict keys; the computation runs on libdamvs's fused NHWC conv2d kernels
(frontend_hip.py, BN folded by frontend_fold.py), whose outputs already have the NHWC layout the
warp/aggregation kernel reads. ``frontend_impl="torch"`` keeps a PyTorch-ROCm (MIOpen) channels-last path
for A/B comparisons only.

The module trees reproduce the reference's ``state_dict`` keys exactly so that
``load_state_dict(torch.load(ckpt)['model'], strict=True)`` (test_uni.py:223-224) works:

* ``FeatureNet``          models/module.py:355-462  (fpn and unet arch modes)
* ``GeoFeatureFusion``    models/geometry.py:14-277 ("z" encoding, "basic" mask, add_origin_feat)
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class ConvBNReLU2d(nn.Module):
    """conv(bias=False) -> BN -> ReLU with attribute names ``conv``/``bn`` (module.py:28-66)."""

    def __init__(self, cin, cout, k, stride=1, padding=0, relu=True):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, stride=stride, padding=padding, bias=False)
        self.bn = nn.BatchNorm2d(cout, momentum=0.1)
        self.relu = relu

    def forward(self, x):
        x = self.bn(self.conv(x))
        return F.relu(x) if self.relu else x


class DeconvBNReLU2d(nn.Module):
    """ConvTranspose2d -> crop to 2x -> BN -> ReLU (module.py:69-115)."""

    def __init__(self, cin, cout, k, stride=1, **kw):
        super().__init__()
        self.conv = nn.ConvTranspose2d(cin, cout, k, stride=stride, bias=False, **kw)
        self.bn = nn.BatchNorm2d(cout, momentum=0.1)
        self.stride = stride

    def forward(self, x):
        y = self.conv(x)
        if self.stride == 2:
            y = y[:, :, :2 * x.shape[2], :2 * x.shape[3]].contiguous()
        return F.relu(self.bn(y))


class FuseUp2d(nn.Module):
    """unet-mode decoder step: deconv x2, concat skip, conv (module.py:334-352)."""

    def __init__(self, cin, cout, k):
        super().__init__()
        self.deconv = DeconvBNReLU2d(cin, cout, k, stride=2, padding=1, output_padding=1)
        self.conv = ConvBNReLU2d(2 * cout, cout, k, 1, padding=1)

    def forward(self, skip, x):
        return self.conv(torch.cat((self.deconv(x), skip), dim=1))


class FeatureNet(nn.Module):
    """Three-level feature pyramid; outputs stage1 (C=32, 1/4), stage2 (16, 1/2), stage3 (8, 1)."""

    def __init__(self, base_channels=8, num_stage=3, stride=4, arch_mode="fpn"):
        super().__init__()
        assert arch_mode in ("unet", "fpn"), arch_mode
        b = base_channels
        self.arch_mode, self.num_stage, self.stride, self.base_channels = arch_mode, num_stage, stride, b
        cbr = ConvBNReLU2d
        self.conv0 = nn.Sequential(cbr(3, b, 3, 1, 1), cbr(b, b, 3, 1, 1))
        self.conv1 = nn.Sequential(cbr(b, 2 * b, 5, 2, 2), cbr(2 * b, 2 * b, 3, 1, 1), cbr(2 * b, 2 * b, 3, 1, 1))
        self.conv2 = nn.Sequential(cbr(2 * b, 4 * b, 5, 2, 2), cbr(4 * b, 4 * b, 3, 1, 1), cbr(4 * b, 4 * b, 3, 1, 1))
        self.out1 = nn.Conv2d(4 * b, 4 * b, 1, bias=False)
        self.out_channels = [4 * b]
        if arch_mode == "unet":
            self.deconv1 = FuseUp2d(4 * b, 2 * b, 3)
            self.out2 = nn.Conv2d(2 * b, 2 * b, 1, bias=False)
            self.out_channels.append(2 * b)
            if num_stage == 3:
                self.deconv2 = FuseUp2d(2 * b, b, 3)
                self.out3 = nn.Conv2d(b, b, 1, bias=False)
                self.out_channels.append(b)
        else:
            self.inner1 = nn.Conv2d(2 * b, 4 * b, 1, bias=True)
            if num_stage == 3:
                self.inner2 = nn.Conv2d(b, 4 * b, 1, bias=True)
                self.out2 = nn.Conv2d(4 * b, 2 * b, 3, padding=1, bias=False)
                self.out3 = nn.Conv2d(4 * b, b, 3, padding=1, bias=False)
                self.out_channels += [2 * b, b]
            else:
                self.out2 = nn.Conv2d(4 * b, b, 3, padding=1, bias=False)
                self.out_channels.append(b)

    def forward(self, x):
        c0 = self.conv0(x.to(self.out1.weight.dtype))
        c1 = self.conv1(c0)
        c2 = self.conv2(c1)
        out = {"stage1": self.out1(c2)}
        if self.arch_mode == "unet":
            f = self.deconv1(c1, c2)
            out["stage2"] = self.out2(f)
            if self.num_stage == 3:
                out["stage3"] = self.out3(self.deconv2(c0, f))
        else:
            f = F.interpolate(c2, scale_factor=2, mode="nearest") + self.inner1(c1)
            out["stage2"] = self.out2(f)
            if self.num_stage == 3:
                f = F.interpolate(f, scale_factor=2, mode="nearest") + self.inner2(c0)
                out["stage3"] = self.out3(f)
        return out


def _cbr(cin, cout, k, s, p):
    """models/geometry.py:467-472 (Sequential: 0 conv, 1 BN, 2 ReLU)."""
    return nn.Sequential(nn.Conv2d(cin, cout, k, stride=s, padding=p, bias=False), nn.BatchNorm2d(cout), nn.ReLU())


def _dbr(cin, cout, k, s, p, op):
    """models/geometry.py:475-480 (Sequential: 0 ConvTranspose2d, 1 BN, 2 ReLU)."""
    return nn.Sequential(nn.ConvTranspose2d(cin, cout, k, stride=s, padding=p, output_padding=op, bias=False),
                         nn.BatchNorm2d(cout), nn.ReLU())


class GeoBlock(nn.Module):
    """Residual block whose convs see an extra depth plane (models/geometry.py:381-433)."""

    def __init__(self, cin, cout, stride=1, geo=1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin + geo, cout, 3, stride=stride, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout + geo, cout, 3, stride=1, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin + geo, cout, 1, stride=stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x, g1, g2):
        xg = torch.cat((x, g1), 1)
        y = F.relu(self.bn1(self.conv1(xg)))
        y = self.bn2(self.conv2(torch.cat((g2, y), 1)))
        idt = self.downsample(xg) if self.downsample is not None else x
        return F.relu(y + idt)


def sparse_pool_close(d, mask, big=600.0):
    """SparseDownSampleClose(stride=2) (models/geometry.py:443-455): keep the closest valid depth."""
    enc = -(1 - mask) * big - d
    dd = -F.max_pool2d(enc, 2, 2)
    m = F.max_pool2d(mask, 2, 2)
    return dd - (1 - m) * big, m


class GeoFeatureFusion(nn.Module):
    """RGB + previous-stage-depth encoder/decoder that replaces the reference feature at stages 2/3."""

    # (name, kind, args) in registration order so that state_dict keys and order match the reference.
    _SPEC = (
        ("rgb_conv_init", "cbr", (4, 8, 5, 1, 2)),
        ("rgb_encoder_layer1", "geo", (8, 16, 2)), ("rgb_encoder_layer2", "geo", (16, 32, 1)),
        ("rgb_encoder_layer3", "geo", (32, 64, 2)), ("rgb_encoder_layer4", "geo", (64, 128, 1)),
        ("rgb_encoder_layer5", "geo", (128, 256, 2)),
        ("rgb_decoder_layer4", "dbr", (256, 128, 5, 2, 2, 1)), ("rgb_decoder_layer2", "dbr", (128, 32, 5, 2, 2, 1)),
        ("rgb_decoder_layer0", "dbr", (32, 16, 3, 1, 1, 0)), ("rgb_decoder_layer", "dbr", (16, 8, 5, 2, 2, 1)),
        ("rgb_decoder_output", "dbr", (8, 2, 3, 1, 1, 0)),
        ("depth_conv_init", "cbr", (2, 8, 5, 1, 2)),
        ("depth_layer1", "geo", (8, 16, 2)), ("depth_layer2", "geo", (16, 32, 1)),
        ("depth_layer3", "geo", (64, 64, 2)), ("depth_layer4", "geo", (64, 128, 1)),
        ("depth_layer5", "geo", (256, 256, 2)),
        ("decoder_layer3", "dbr", (256, 128, 5, 2, 2, 1)), ("decoder_layer4", "dbr", (128, 64, 3, 1, 1, 0)),
        ("decoder_layer5", "dbr", (64, 32, 5, 2, 2, 1)), ("decoder_layer6", "dbr", (32, 16, 3, 1, 1, 0)),
        ("decoder_layer7", "dbr", (16, 8, 5, 2, 2, 1)),
        ("rgbdepth_decoder_stage1", "dbr", (32, 32, 5, 2, 2, 1)), ("rgbdepth_decoder_stage2", "dbr", (16, 16, 5, 2, 2, 1)),
        ("rgbdepth_decoder_stage3", "dbr", (8, 8, 3, 1, 1, 0)),
        ("final_decoder_stage1", "dbr", (32, 32, 3, 1, 1, 0)), ("final_decoder_stage2", "dbr", (16, 16, 3, 1, 1, 0)),
        ("final_decoder_stage3", "dbr", (8, 8, 3, 1, 1, 0)),
    )

    def __init__(self, convolutional_layer_encoding="z", mask_type="basic", add_origin_feat_flag=True):
        super().__init__()
        if convolutional_layer_encoding != "z" or mask_type not in ("basic", "mean"):
            raise NotImplementedError("only the reference's active configuration ('z' encoding) is supported")
        self.convolutional_layer_encoding = convolutional_layer_encoding
        self.mask_type = mask_type
        self.add_origin_feat_flag = add_origin_feat_flag
        for name, kind, a in self._SPEC:
            mod = {"cbr": lambda: _cbr(*a), "dbr": lambda: _dbr(*a), "geo": lambda: GeoBlock(*a)}[kind]()
            setattr(self, name, mod)

    def forward(self, rgb, depth, confidence, depth_values, stage_idx, origin_feat, intrinsics_matrices_stage=None):
        dmin = depth_values[:, 0, None, None, None]
        dmax = depth_values[:, -1, None, None, None]
        d = (depth - dmin) / (dmax - dmin)
        if self.mask_type == "basic":
            vm = (d > 0).to(d.dtype)
        else:
            vm = torch.logical_and(d > 0, confidence > confidence.mean()).to(d.dtype)
        d2, m2 = sparse_pool_close(d, vm)
        d3, m3 = sparse_pool_close(d2, m2)
        d4, _ = sparse_pool_close(d3, m3)
        wd = self.rgb_conv_init[0].weight.dtype  # geometry in fp32, convs in the module's dtype
        rgb, d, d2, d3, d4 = (t.to(wd) for t in (rgb, d, d2, d3, d4))
        origin_feat = origin_feat.to(wd)

        r0 = self.rgb_conv_init(torch.cat((rgb, d), 1))
        r1 = self.rgb_encoder_layer1(r0, d, d2)
        r2 = self.rgb_encoder_layer2(r1, d2, d2)
        r3 = self.rgb_encoder_layer3(r2, d2, d3)
        r4 = self.rgb_encoder_layer4(r3, d3, d3)
        r5 = self.rgb_encoder_layer5(r4, d3, d4)
        r4p = self.rgb_decoder_layer4(r5) + r4
        r2p = self.rgb_decoder_layer2(r4p) + r2
        r0p = self.rgb_decoder_layer0(r2p) + r1
        rp = self.rgb_decoder_layer(r0p) + r0
        rgb_out = self.rgb_decoder_output(rp)

        s0 = self.depth_conv_init(torch.cat((d, rgb_out[:, 0:1]), 1))
        s1 = self.depth_layer1(s0, d, d2)
        s2 = self.depth_layer2(s1, d2, d2)
        s3 = self.depth_layer3(torch.cat([r2p, s2], 1), d2, d3)
        s4 = self.depth_layer4(s3, d3, d3)
        s5 = self.depth_layer5(torch.cat([r4p, s4], 1), d3, d4)

        dec4 = self.decoder_layer4(s4 + self.decoder_layer3(r5 + s5))
        dec6 = self.decoder_layer6(self.decoder_layer5(dec4))
        if stage_idx == 1:
            f = self.rgbdepth_decoder_stage2(s1 + dec6)
            return self.final_decoder_stage2(f + origin_feat if self.add_origin_feat_flag else f)
        if stage_idx == 2:
            f = self.rgbdepth_decoder_stage3(s0 + self.decoder_layer7(dec6))
            return self.final_decoder_stage3(f + origin_feat if self.add_origin_feat_flag else f)
        raise ValueError("GeoFeatureFusion runs at stage_idx 1 or 2, got %r" % (stage_idx,))
