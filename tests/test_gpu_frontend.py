"""GPU: the HIP 2D front-end (damvs_conv2d_*) against plain PyTorch fp32 references and the oracle.

Layer level: every form the front-end uses (conv k1/k3/k5 s1/s2, transposed k3 s1 / k5 s2, two
concatenated tensor inputs, fp32 planar inputs at any weight channel, residual before / after ReLU,
nearest-x2 upsampled residual, channel padding of cout=2) vs F.conv2d / F.conv_transpose2d on the
explicitly concatenated input. Network level: FeatureNet and GeoFeatureFusion vs the oracle.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from conftest import rel_max
from common import model_state, forward_inputs
from oracle import mvs_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from damvsnet_amd import build, _capi
    build.build()
    _capi.load_library()


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


# (transposed, k, s, p, op, c0, c1, geo positions, cout, relu, pre, post_up)
CASES = [
    (False, 3, 1, 1, 0, 16, 0, (), 32, True, False, 0),
    (False, 5, 2, 2, 0, 8, 0, (), 16, True, False, 0),
    (False, 1, 2, 0, 0, 16, 0, (16,), 32, False, False, 0),          # GeoBlock downsample
    (False, 3, 2, 1, 0, 32, 32, (64,), 64, True, False, 0),         # cat([a, b], g1) conv1
    (False, 3, 1, 1, 0, 16, 0, (0,), 16, True, True, 0),            # cat(g2, y) conv2 + identity
    (False, 5, 1, 2, 0, 0, 0, (0, 1, 2, 3), 8, True, False, 0),      # rgb_conv_init (4 planes)
    (False, 3, 1, 1, 0, 0, 0, (0, 1, 2), 12, False, True, 2),        # planes-only, cout 12, both residuals
    (False, 3, 2, 1, 0, 0, 0, (0, 1), 2, True, False, 0),            # planes-only, stride 2, cout 2
    (False, 1, 1, 0, 0, 16, 0, (), 32, False, False, 2),            # FPN inner conv + up2 residual
    (True, 5, 2, 2, 1, 64, 0, (), 32, True, False, 1),              # decoder deconv + skip
    (True, 3, 1, 1, 0, 16, 0, (), 8, True, False, 1),
    (True, 3, 1, 1, 0, 8, 0, (), 2, True, False, 0),                # rgb_decoder_output (cout 2)
    (False, 3, 1, 1, 0, 256, 0, (), 256, True, False, 0),           # wide layer (cout tiling)
    (False, 3, 1, 1, 0, 32, 32, (64,), 64, True, True, 0),          # two inputs + plane (wide, 64-channel block)
    (True, 5, 2, 2, 1, 128, 0, (), 32, True, False, 1),             # halo kernel: k5 s2 phases, cout 32
    (True, 3, 1, 1, 0, 64, 0, (), 128, True, True, 0),              # halo kernel: transposed k3 s1, MT 8
    (True, 4, 2, 1, 0, 16, 0, (), 8, False, False, 0),              # x-pair phases: FPN top (k4 s2), cout 8
    (True, 5, 2, 2, 1, 16, 0, (), 8, True, True, 2),                # x-pair + both residuals (post up 2)
    (True, 3, 2, 1, 1, 16, 16, (), 8, True, False, 1),              # x-pair, two inputs
    (False, 3, 1, 1, 0, 128, 0, (0,), 128, True, True, 0),          # wide kernel: GeoBlock conv2 (plane first)
    (False, 3, 1, 1, 0, 128, 128, (256,), 256, True, True, 2),      # wide: two inputs + plane, both residuals
    (True, 5, 2, 2, 1, 256, 0, (), 128, True, False, 1),            # wide: k5 s2 transposed decoder + skip
    (False, 1, 1, 0, 0, 64, 0, (64,), 128, False, False, 0),        # wide: 1x1 (GeoBlock downsample)
    (False, 3, 1, 1, 0, 32, 0, (0,), 32, True, True, 0),            # halo, one slice (bf16): 32+g -> 32
    (False, 3, 1, 1, 0, 32, 0, (32,), 16, True, False, 0),          # halo, one slice, one cout tile
    (False, 3, 1, 1, 0, 0, 0, (0, 1, 2), 8, True, False, 0),         # planes: FeatureNet RGB conv 3->8
    (False, 5, 1, 2, 0, 0, 0, (0, 1), 8, True, False, 0),            # planes: depth_conv_init 2->8
    # wide kernel at input stride 2 (GeoBlock conv1 of the 128 -> 256 levels), ragged q-tiles and an odd width
    (False, 3, 2, 1, 0, 128, 128, (256,), 256, True, False, 0, (37, 151)),
    (False, 3, 2, 1, 0, 128, 0, (128,), 256, True, False, 0, (20, 24)),
    (False, 3, 2, 1, 0, 64, 32, (0,), 128, False, True, 0, (30, 260)),
    # wide kernel's 64-channel block (4 x 64 q-tiles): GeoBlock 64+g -> 64, transposed k3 s1 128 -> 64
    (False, 3, 1, 1, 0, 64, 0, (64,), 64, True, True, 0, (37, 151)),
    (True, 3, 1, 1, 0, 128, 0, (), 64, True, False, 0, (30, 70)),
    # 64-channel block at input stride 2 (2 x 64 q-tiles, 32-column waves): GeoBlock conv1 32+32+g -> 64, 32+g -> 64
    (False, 3, 2, 1, 0, 32, 32, (64,), 64, True, False, 0, (37, 151)),
    (False, 3, 2, 1, 0, 32, 0, (32,), 64, True, True, 0, (64, 130)),
    # LDS-tiled 3x3 kernel with the GeoBlock depth plane (round 6): cat(g, y) 16+g -> 16, cat(x, g) 16+g -> 32, ragged
    (False, 3, 1, 1, 0, 16, 0, (0,), 16, True, True, 0, (37, 151)),
    (False, 3, 1, 1, 0, 16, 0, (16,), 32, True, False, 0, (20, 70)),
    (False, 3, 1, 1, 0, 8, 0, (8,), 16, False, False, 2, (22, 64)),
    # stride-2 5x5 LDS kernel (FeatureNet conv1.0 / conv2.0): ragged tiles, odd sizes, residual, cout 16 / 32
    (False, 5, 2, 2, 0, 8, 0, (), 16, True, False, 0, (70, 262)),
    (False, 5, 2, 2, 0, 16, 0, (), 32, True, False, 0, (37, 151)),
    (False, 5, 2, 2, 0, 16, 0, (), 16, False, True, 0, (30, 66)),
    (False, 5, 2, 2, 0, 8, 0, (), 32, True, True, 0, (9, 17)),
]


@pytest.mark.parametrize("case", CASES, ids=[str(i) for i in range(len(CASES))])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv2d_layer_vs_torch(case, dtype):
    from damvsnet_amd.frontend_hip import HipConv2d, planes
    tr, k, s, p, op, c0, c1, geo, cout, relu, pre, post_up = case[:12]
    g = torch.Generator().manual_seed(hash(case) % 1000)
    B, (H, W) = 2, (case[12] if len(case) > 12 else (20, 24))
    cin = c0 + c1 + len(geo)
    conv = (nn.ConvTranspose2d(cin, cout, k, stride=s, padding=p, output_padding=op) if tr
            else nn.Conv2d(cin, cout, k, stride=s, padding=p))
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.2)
        conv.bias.copy_(torch.randn(conv.bias.shape, generator=g) * 0.1)
    a = torch.randn(B, c0, H, W, generator=g) if c0 else None
    b = torch.randn(B, c1, H, W, generator=g) if c1 else None
    gp = torch.randn(B, len(geo), H, W, generator=g) if geo else None
    # assemble the reference input in weight-channel order
    full = torch.zeros(B, cin, H, W)
    tensor_at = [c for c in range(cin) if c not in geo]
    if c0:
        full[:, tensor_at[:c0]] = a
    if c1:
        full[:, tensor_at[c0:]] = b
    for i, gc in enumerate(geo):
        full[:, gc] = gp[:, i]
    if dtype == torch.bfloat16:  # tensor inputs are stored in bf16
        full[:, tensor_at] = full[:, tensor_at].to(dtype).float()
    ref = conv(full)
    res_pre = torch.randn(ref.shape, generator=g) if pre else None
    post = None
    if post_up:
        post = torch.randn(B, cout, ref.shape[2] // post_up, ref.shape[3] // post_up, generator=g)
    if dtype == torch.bfloat16:
        res_pre = res_pre.to(dtype).float() if res_pre is not None else None
        post = post.to(dtype).float() if post is not None else None
    y = ref + (res_pre if res_pre is not None else 0)
    y = F.relu(y) if relu else y
    if post is not None:
        y = y + F.interpolate(post, scale_factor=post_up, mode="nearest")
    at = dict(c0=c0, c1=c1, c1_at=0)
    if c0 and c1:
        at = dict(c0=c0, c0_at=tensor_at[0], c1=c1, c1_at=tensor_at[c0])
    elif c0:
        at = dict(c0=c0, c0_at=tensor_at[0])
    L = HipConv2d(conv, dtype, relu, geo_at=geo, **at)
    cs = L.cout_store
    padc = lambda t: F.pad(t, (0, 0, 0, 0, 0, cs - cout)) if t is not None and cs != cout else t
    out = L(B, H, W, nhwc(a).to(DEV, dtype) if c0 else None, nhwc(b).to(DEV, dtype) if c1 else None,
            geo=planes(gp.to(DEV)) if geo else (),
            res_pre=nhwc(padc(res_pre)).to(DEV, dtype) if pre else None,
            res_post=nhwc(padc(post)).to(DEV, dtype) if post_up else None, post_up=max(post_up, 1))
    got = out.float().cpu()[..., :cout].permute(0, 3, 1, 2)
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    assert got.shape == y.shape
    assert rel_max(got.numpy(), y.detach().numpy()) < tol


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-5), (torch.bfloat16, 3e-2)])
def test_fpn_top_reassociation_vs_torch(dtype, tol):
    """out3(up2(f) + inner2(c0)) (models/module.py:455-459) against fpn_top_layers' re-associated form:
    transposed sum-of-taps conv of f + composed 3x3 conv of c0 + full-sum bias with the border fix-up
    (damvs_conv2d_border_bias) — every border pixel and corner included."""
    from damvsnet_amd import _capi
    from damvsnet_amd.engine import DTYPES
    from damvsnet_amd.frontend_hip import fpn_top_layers
    g = torch.Generator().manual_seed(3)
    inner2, out3 = nn.Conv2d(8, 32, 1, bias=True), nn.Conv2d(32, 8, 3, padding=1, bias=False)
    with torch.no_grad():
        for m in (inner2, out3):
            m.weight.copy_(torch.randn(m.weight.shape, generator=g) * 0.2)
        inner2.bias.copy_(torch.randn(32, generator=g))
    B, H, W = 2, 12, 20
    c0 = torch.randn(B, 8, H, W, generator=g)
    f = torch.randn(B, 32, H // 2, W // 2, generator=g)
    if dtype == torch.bfloat16:
        c0, f = c0.to(dtype).float(), f.to(dtype).float()
    ref = out3(F.interpolate(f, scale_factor=2, mode="nearest") + inner2(c0)).detach()
    up, conv, corr, _ = fpn_top_layers(inner2, out3, dtype)
    t = up(B, H // 2, W // 2, nhwc(f).to(DEV, dtype))
    o = conv(B, H, W, nhwc(c0).to(DEV, dtype), res_pre=t)
    lib = _capi.load_library()
    _capi.check(lib.damvs_conv2d_border_bias(_capi.stream_ptr(o.device), DTYPES[dtype], B, H, W, o.shape[3], 8,
                                             _capi.float_ptr(corr), o.data_ptr()))
    got = o.float().cpu().permute(0, 3, 1, 2)
    assert rel_max(got.numpy(), ref.numpy()) < tol
    # argument checks: cout beyond the 16-channel table, null output
    with pytest.raises(_capi.DamvsError):
        _capi.check(lib.damvs_conv2d_border_bias(_capi.stream_ptr(o.device), DTYPES[dtype], B, H, W, 32, 17,
                                                 _capi.float_ptr(torch.zeros(9 * 17)), o.data_ptr()))
    with pytest.raises(_capi.DamvsError):
        _capi.check(lib.damvs_conv2d_border_bias(_capi.stream_ptr(o.device), DTYPES[dtype], B, H, W, 8, 8,
                                                 _capi.float_ptr(corr), None))


def _folded(sd, dtype):
    from damvsnet_amd.cascade import CascadeMVSNet
    from damvsnet_amd.frontend_fold import fold_frontend
    net = CascadeMVSNet(ndepths=[48, 32, 8])
    net.load_state_dict(sd)
    return (fold_frontend(net.feature, torch.float32).to(DEV), fold_frontend(net.GeoFeatureFusionNet, torch.float32).to(DEV))


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 5e-2)])
def test_featurenet_hip_vs_oracle(dtype, tol):
    from damvsnet_amd.frontend_hip import HipFeatureNet
    sd = model_state("forward_160x128_48_32_8")
    fnet, _ = _folded(sd, dtype)
    imgs, _, _, _ = forward_inputs(1, 5, 128, 160)
    x = imgs[0]  # 5 views as a batch
    ref = O.feature_net(x, sd)
    got = HipFeatureNet(fnet, dtype)(x.to(DEV))
    for k in ("stage1", "stage2", "stage3"):
        err = rel_max(got[k].float().cpu().permute(0, 3, 1, 2).numpy(), ref[k].numpy())
        assert err < tol, (k, err)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 5e-2)])
def test_featurenet_unet_hip_vs_reference(dtype, tol):
    """arch_mode="unet" FeatureNet (models/module.py:385-399,430-441; DeConv2dFuse :334-352) on the HIP
    front-end against the reference's own outputs (tests/golden/featurenet_unet.npz) and the oracle."""
    from common import featurenet_unet_state
    from conftest import golden
    from damvsnet_amd import synth
    from damvsnet_amd.frontend import FeatureNet
    from damvsnet_amd.frontend_fold import fold_frontend
    from damvsnet_amd.frontend_hip import HipFeatureNet
    sd = featurenet_unet_state()
    net = FeatureNet(base_channels=8, stride=4, num_stage=3, arch_mode="unet")
    net.load_state_dict(sd, strict=True)
    x = torch.from_numpy(synth.images(1, 2, 96, 128, seed=0)[0])
    g = golden("featurenet_unet")
    ref = O.feature_net(x, {"feature." + k: v for k, v in sd.items()}, arch_mode="unet")
    got = HipFeatureNet(fold_frontend(net, torch.float32).to(DEV), dtype)(x.to(DEV))
    for k in ("stage1", "stage2", "stage3"):
        y = got[k].float().cpu().permute(0, 3, 1, 2).numpy()
        assert rel_max(y, g[k]) < tol and rel_max(y, ref[k].numpy()) < tol, k


@pytest.mark.parametrize("stage_idx", [1, 2])
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 8e-2)])
def test_geofusion_hip_vs_oracle(stage_idx, dtype, tol):
    from damvsnet_amd.frontend_hip import HipGeoFeatureFusion
    sd = model_state("forward_160x128_48_32_8")
    _, geo = _folded(sd, dtype)
    imgs, _, dv, _ = forward_inputs(2, 5, 128, 160)
    g = torch.Generator().manual_seed(stage_idx)
    scale = 2 ** (2 - stage_idx)
    h, w = 128 // scale, 160 // scale
    C = (32, 16, 8)[stage_idx]
    rgb = F.interpolate(imgs[:, 0], size=(h, w), mode="bilinear", align_corners=False)
    depth = 425 + 500 * torch.rand(2, 1, h, w, generator=g)
    depth[:, :, :4] = 300.0  # invalid (d <= 0) rows exercise the sparse-pool mask
    conf = torch.rand(2, 1, h, w, generator=g)
    origin = torch.randn(2, C, h, w, generator=g)
    ref = O.geo_feature_fusion(rgb, depth, conf, dv, stage_idx, origin, sd)
    got = HipGeoFeatureFusion(geo, dtype)(rgb.to(DEV), depth.to(DEV), conf.to(DEV), dv.to(DEV), stage_idx,
                                           nhwc(origin).to(DEV, dtype))
    err = rel_max(got.float().cpu().permute(0, 3, 1, 2).numpy(), ref.numpy())
    assert err < tol, err


@pytest.mark.parametrize("hw", [(64, 80), (37, 51), (8, 9)])
@pytest.mark.parametrize("mask_type", ["basic", "mean"])
def test_sparse_depth_pyramid_bitwise_vs_torch(hw, mask_type):
    """damvs_sparse_depth_pyramid vs the reference's own torch ops (models/geometry.py:90-96 normalisation
    and mask, SparseDownSampleClose :443-455 three times) on the GPU: bitwise, odd sizes included."""
    from damvsnet_amd.frontend import sparse_pool_close
    from damvsnet_amd.frontend_hip import sparse_depth_pyramid
    h, w = hw
    g = torch.Generator().manual_seed(h * w)
    depth = (425 + 500 * torch.rand(3, 1, h, w, generator=g)).to(DEV)
    depth[:, :, : h // 3] = 300.0                                 # invalid rows (d <= 0)
    depth[1, 0, :, 1::3] = 200.0                                  # ragged invalid columns
    conf = torch.rand(3, 1, h, w, generator=g).to(DEV)
    dv = torch.stack([torch.linspace(425, 935, 48), torch.linspace(400, 900, 48),
                      torch.linspace(500, 1000, 48)]).to(DEV)
    dmin, dmax = dv[:, 0, None, None, None], dv[:, -1, None, None, None]
    d = (depth - dmin) / (dmax - dmin)
    if mask_type == "basic":
        vm, mask = torch.where(d > 0, torch.full_like(d, 1.0), torch.full_like(d, 0.0)), None
    else:
        vm = torch.where(torch.logical_and(d > 0, conf > conf.mean()), torch.full_like(d, 1.0), torch.full_like(d, 0.0))
        mask = vm
    d2, m2 = sparse_pool_close(d, vm)
    d3, m3 = sparse_pool_close(d2, m2)
    d4, _ = sparse_pool_close(d3, m3)
    got = sparse_depth_pyramid(depth, dv, mask)
    for lvl, (a, b) in enumerate(zip(got, (d, d2, d3, d4))):
        assert a.shape == b.shape, (lvl, a.shape, b.shape)
        assert torch.equal(a, b), (lvl, (a - b).abs().max().item())


def test_featurenet_views_read_in_place():
    """A (B, N, 3, H, W) batch goes through HipFeatureNet with the first layer reading each view's
    planes in place (no view-major copy of the images): bitwise equal to the copied batch."""
    from damvsnet_amd.frontend_hip import HipFeatureNet
    sd = model_state("forward_160x128_48_32_8")
    fnet, _ = _folded(sd, torch.bfloat16)
    net = HipFeatureNet(fnet, torch.bfloat16)
    imgs, _, _, _ = forward_inputs(2, 3, 64, 96)
    imgs = imgs.to(DEV)
    B, N = imgs.shape[:2]
    a = net(imgs)
    b = net(imgs.transpose(0, 1).reshape(N * B, *imgs.shape[2:]))
    for k in a:
        assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_featurenet_view_groups_bitwise(dtype, monkeypatch):
    """Views in groups (HipFeatureNet.MAX_ACT_BYTES: the 2 GiB operand bound at cfgE's fp32 B=4) give the one-call
    result bitwise: every layer is per-image, and the groups' outputs are concatenated in view order. The bound is
    lowered here so that 5 views run as groups of 2, 2, 1."""
    from damvsnet_amd.frontend_hip import HipFeatureNet
    sd = model_state("forward_160x128_48_32_8")
    fnet, _ = _folded(sd, dtype)
    net = HipFeatureNet(fnet, dtype)
    imgs, _, _, _ = forward_inputs(2, 5, 64, 96)
    imgs = imgs.to(DEV)
    a = net(imgs)
    per_view = 2 * 64 * 96 * 8 * torch.tensor([], dtype=dtype).element_size()
    monkeypatch.setattr(HipFeatureNet, "MAX_ACT_BYTES", 2 * per_view + 1)
    b = net(imgs)
    assert a.keys() == b.keys()
    for k in a:
        assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("dt,tol", [(torch.bfloat16, 3e-2), (torch.float32, 2e-5)])
@pytest.mark.parametrize("B,H,W", [(2, 12, 20), (1, 40, 260), (3, 18, 134)])
def test_fpn_top_fused_vs_torch(B, H, W, dt, tol):
    """damvs_fpn_top_forward (the 3x3 conv of c0 and the transposed conv of f in one launch, x-pair MFMA
    layout) + border fix-up vs out3(up2(f) + inner2(c0)) in fp32 torch (models/module.py:455-459), on
    partial tiles in both directions, and vs the two-launch path. fp32: damvs_fpn_top_forward_f32 (split-f16
    MFMAs, 4-row tiles), at fp32 tolerance."""
    from damvsnet_amd import _capi
    from damvsnet_amd.engine import DTYPES
    from damvsnet_amd.frontend_hip import fpn_top_layers, pack_fpn_top, pack_fpn_top_split
    g = torch.Generator().manual_seed(H * W)
    inner2, out3 = nn.Conv2d(8, 32, 1, bias=True), nn.Conv2d(32, 8, 3, padding=1, bias=False)
    with torch.no_grad():
        for m in (inner2, out3):
            m.weight.copy_(torch.randn(m.weight.shape, generator=g) * 0.2)
        inner2.bias.copy_(torch.randn(32, generator=g))
    c0 = torch.randn(B, 8, H, W, generator=g).to(dt).float()
    f = torch.randn(B, 32, H // 2, W // 2, generator=g).to(dt).float()
    ref = out3(F.interpolate(f, scale_factor=2, mode="nearest") + inner2(c0)).detach()
    up, conv, corr, (wt, wc, bc) = fpn_top_layers(inner2, out3, dt)
    lib = _capi.load_library()
    c0d, fd = nhwc(c0).to(DEV, dt), nhwc(f).to(DEV, dt)
    o = torch.empty(B, H, W, 8, device=DEV, dtype=dt)
    bd = bc.float().to(DEV)
    if dt == torch.bfloat16:
        ap = pack_fpn_top(wt, wc).to(DEV)  # held until the launch has run
        _capi.check(lib.damvs_fpn_top_forward(_capi.stream_ptr(o.device), B, H, W, c0d.data_ptr(), fd.data_ptr(),
                                              ap.data_ptr(), bd.data_ptr(), o.data_ptr()))
    else:
        ap, ws = pack_fpn_top_split(wt, wc)
        ap = ap.to(DEV)
        _capi.check(lib.damvs_fpn_top_forward_f32(_capi.stream_ptr(o.device), B, H, W, c0d.data_ptr(), fd.data_ptr(),
                                                  ap.data_ptr(), ws, bd.data_ptr(), o.data_ptr()))
    o2 = conv(B, H, W, c0d, res_pre=up(B, H // 2, W // 2, fd))
    for t in (o, o2):
        _capi.check(lib.damvs_conv2d_border_bias(_capi.stream_ptr(t.device), DTYPES[dt], B, H, W, 8, 8,
                                                 _capi.float_ptr(corr), t.data_ptr()))
    got = o.float().cpu().permute(0, 3, 1, 2)
    e1, e2 = rel_max(got.numpy(), ref.numpy()), rel_max(got.numpy(), o2.float().cpu().permute(0, 3, 1, 2).numpy())
    print("fpn_top fused %s: vs torch %.2e, vs two launches %.2e" % (dt, e1, e2))
    assert e1 < tol and e2 < tol
    with pytest.raises(_capi.DamvsError):  # odd sizes are refused
        _capi.check(lib.damvs_fpn_top_forward(_capi.stream_ptr(o.device), B, H - 1, W, c0d.data_ptr(),
                                              fd.data_ptr(), fd.data_ptr(), fd.data_ptr(), o.data_ptr()))


@pytest.mark.parametrize("k,ng,relu,pre", [(5, 4, True, False), (5, 2, True, True), (5, 1, False, False)])
def test_planes_four_columns_bitwise(k, ng, relu, pre, monkeypatch):
    """The 4-column plane-only kernel (conv2d_planes4_kernel: FeatureNet's RGB conv, GeoFF's RGB+depth and depth init
    convs) against the one-column kernel it replaces: same fused multiply-adds per output, so bitwise equal (odd H,
    first / last column groups at the image edges, with and without a residual)."""
    from damvsnet_amd.frontend_hip import HipConv2d, planes
    g = torch.Generator().manual_seed(7 * k + ng)
    B, H, W, cout = 2, 21, 36, 8
    conv = nn.Conv2d(ng, cout, k, padding=k // 2)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.2)
        conv.bias.copy_(torch.randn(conv.bias.shape, generator=g) * 0.1)
    gp = planes(torch.randn(B, ng, H, W, generator=g).to(DEV))
    res = torch.randn(B, H, W, cout, generator=g).to(DEV, torch.bfloat16) if pre else None
    L = HipConv2d(conv, torch.bfloat16, relu, geo_at=tuple(range(ng)), c0=0, c1=0, c1_at=0)
    monkeypatch.setenv("DAMVS_PLANES_MFMA", "0")  # the VALU kernels (the MFMA form takes these layers by default)
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("DAMVS_PLANES4", flag)
        outs.append(L(B, H, W, None, None, geo=gp, res_pre=res).clone())
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


# The LDS-tiled 3x3 kernel with a depth plane (conv2d_lds_kernel, round 6) against the gather kernel it replaces
# (DAMVS_CONV2D_LDS_PLANE=0): the same MFMA sequence per accumulator (tensor chunks, then the plane chunk), so bitwise
# equal in bf16 (fp32: the gather kernel is the 32-K form, compared against torch in test_conv2d_layer_vs_torch).
LDS_PLANE_CASES = [
    (16, (0,), 16, True, True, 0, (37, 151)),   # GeoBlock conv2: cat(g2, y) 16+g -> 16, identity residual
    (16, (16,), 32, True, False, 0, (20, 70)),  # GeoBlock conv1 at stride 1: cat(x, g1) 16+g -> 32
    (8, (8,), 16, False, False, 2, (22, 64)),   # 8+g -> 16, upsampled residual after ReLU
]


@pytest.mark.parametrize("case", LDS_PLANE_CASES, ids=[str(i) for i in range(len(LDS_PLANE_CASES))])
def test_lds_plane_bitwise_vs_gather(case, monkeypatch):
    from damvsnet_amd.frontend_hip import HipConv2d, planes
    c0, geo, cout, relu, pre, post_up, (H, W) = case
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(c0 * 7 + cout + H)
    B, cin = 2, c0 + 1
    conv = nn.Conv2d(cin, cout, 3, padding=1)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.2)
        conv.bias.copy_(torch.randn(conv.bias.shape, generator=g) * 0.1)
    x = nhwc(torch.randn(B, c0, H, W, generator=g)).to(DEV, dt)
    gp = planes(torch.randn(B, 1, H, W, generator=g).to(DEV))
    tensor_at = [c for c in range(cin) if c not in geo]
    L = HipConv2d(conv, dt, relu, geo_at=geo, c0=c0, c0_at=tensor_at[0])
    res = torch.randn(B, H, W, L.cout_store, generator=g).to(DEV, dt) if pre else None
    post = torch.randn(B, H // max(post_up, 1), W // max(post_up, 1), L.cout_store, generator=g).to(DEV, dt) \
        if post_up else None
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("DAMVS_CONV2D_LDS_PLANE", flag)
        outs.append(L(B, H, W, x, None, geo=gp, res_pre=res, res_post=post, post_up=max(post_up, 1)).clone())
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


# The LDS-staged x-pair transposed conv (conv2d_xpair_lds_kernel, bf16 and fp32, round 6) against the x-pair gather kernel
# (DAMVS_CONV2D_XPAIR_LDS=0): the same MFMA sequence per accumulator, so bitwise equal. k5 s2 (GeoFF's full-resolution
# decoders) and k4 s2 (FPN top's transposed term), ragged tiles, residuals before / after ReLU.
XPAIR_LDS_CASES = [
    (5, 2, 1, True, True, 2, (37, 151)),
    (5, 2, 1, False, False, 0, (20, 64)),
    (4, 1, 0, False, True, 1, (9, 70)),
]


@pytest.mark.parametrize("case", XPAIR_LDS_CASES, ids=[str(i) for i in range(len(XPAIR_LDS_CASES))])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32], ids=["bf16", "f32"])
def test_xpair_lds_bitwise_vs_gather(case, dt, monkeypatch):
    from damvsnet_amd.frontend_hip import HipConv2d
    k, p, op, relu, pre, post_up, (H, W) = case
    g = torch.Generator().manual_seed(k * 31 + H + W)
    B = 2
    conv = nn.ConvTranspose2d(16, 8, k, stride=2, padding=p, output_padding=op)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.2)
        conv.bias.copy_(torch.randn(conv.bias.shape, generator=g) * 0.1)
    L = HipConv2d(conv, dt, relu, c0=16, c0_at=0)
    Ho, Wo = (H - 1) * 2 - 2 * p + k + op, (W - 1) * 2 - 2 * p + k + op
    x = nhwc(torch.randn(B, 16, H, W, generator=g)).to(DEV, dt)
    res = torch.randn(B, Ho, Wo, L.cout_store, generator=g).to(DEV, dt) if pre else None
    post = torch.randn(B, Ho // max(post_up, 1), Wo // max(post_up, 1), L.cout_store, generator=g).to(DEV, dt) \
        if post_up else None
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("DAMVS_CONV2D_XPAIR_LDS", flag)
        outs.append(L(B, H, W, x, None, res_pre=res, res_post=post, post_up=max(post_up, 1)).clone())
    torch.cuda.synchronize()
    assert outs[0].shape == (B, Ho, Wo, L.cout_store)
    assert torch.equal(outs[0], outs[1])


# The plane-only layers on split-f16 MFMAs (conv2d_planes_mfma_kernel, the default for cout 4 / 8 at Wi % 4 == 0) against
# float64 F.conv2d and against the VALU kernels (DAMVS_PLANES_MFMA=0): FeatureNet's RGB conv (3x3, 3 planes), GeoFF's
# RGB+depth (5x5, 4) and depth+depth (5x5, 2) init convs, 1 plane, cout 4; ragged 16 x 64 tiles (H 37 / 21, W 200 / 36),
# residuals before / after ReLU; plane magnitudes from 1e-6 to 3e4 (the block prescale keeps both f16 pieces normal).
PLANES_MFMA_CASES = [
    (3, 3, 8, True, False, 0, (37, 200), 1.0),
    (5, 4, 8, True, False, 0, (21, 36), 1.0),
    (5, 2, 8, True, True, 0, (37, 200), 1.0),
    (5, 1, 4, False, False, 2, (22, 68), 1.0),
    (3, 3, 8, True, False, 0, (16, 64), 3e4),
    (5, 4, 8, False, False, 0, (21, 36), 1e-6),
]


@pytest.mark.parametrize("case", PLANES_MFMA_CASES, ids=[str(i) for i in range(len(PLANES_MFMA_CASES))])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_planes_mfma_vs_fp64_and_valu(case, dtype, monkeypatch):
    from damvsnet_amd.frontend_hip import HipConv2d, planes
    k, ng, cout, relu, pre, post_up, (H, W), mag = case
    g = torch.Generator().manual_seed(11 * k + ng + cout)
    B = 2
    conv = nn.Conv2d(ng, cout, k, padding=k // 2)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.2)
        conv.bias.copy_(torch.randn(conv.bias.shape, generator=g) * 0.1 * mag)
    x = torch.randn(B, ng, H, W, generator=g) * mag
    gp = planes(x.to(DEV))
    res = torch.randn(B, H, W, cout, generator=g) * mag if pre else None
    post = torch.randn(B, H // max(post_up, 1), W // max(post_up, 1), cout, generator=g) * mag if post_up else None
    if dtype == torch.bfloat16:
        res = res.to(dtype).float() if res is not None else None
        post = post.to(dtype).float() if post is not None else None
    with torch.no_grad():
        ref = F.conv2d(x.double(), conv.weight.double(), conv.bias.double(), padding=k // 2).permute(0, 2, 3, 1)
    ref = ref + res.double() if res is not None else ref
    ref = F.relu(ref) if relu else ref
    if post is not None:
        ref = ref + F.interpolate(post.double().permute(0, 3, 1, 2), scale_factor=post_up, mode="nearest").permute(0, 2, 3, 1)
    L = HipConv2d(conv, dtype, relu, geo_at=tuple(range(ng)), c0=0, c1=0, c1_at=0)
    run = lambda: L(B, H, W, None, None, geo=gp, res_pre=res.to(DEV, dtype) if res is not None else None,
                    res_post=post.to(DEV, dtype) if post is not None else None, post_up=max(post_up, 1)).clone()
    got = run()
    monkeypatch.setenv("DAMVS_PLANES_MFMA", "0")
    valu = run()
    torch.cuda.synchronize()
    got, valu = got.double().cpu()[..., :cout], valu.double().cpu()[..., :cout]
    e64, ev = rel_max(got.numpy(), ref.numpy()), rel_max(got.numpy(), valu.numpy())
    print("planes mfma %s k%d ng%d mag %g: vs fp64 %.2e, vs VALU %.2e" % (dtype, k, ng, mag, e64, ev))
    tol = 2e-6 if dtype == torch.float32 else 1e-2
    assert e64 < tol and ev < (tol if dtype == torch.float32 else 1e-2)


# fp32 wide layers on the rolling K loop (conv2d_wide_kernel RS) against the AG loop (DAMVS_WIDE_RS=0): the same MFMA
# sequence per accumulator, so bitwise equal. Stride-1 128-channel blocks: GeoBlock conv2 with the plane, two inputs +
# plane + both residuals, the k5 s2 transposed decoder (phases of 9 / 6 / 6 / 4 taps), transposed k3 s1, ragged tiles
# (W 70, 130, 200: a last tile column of at most 16 valid q-columns runs one N-group per wave).
RS_CASES = [
    (False, 3, 1, 1, 0, 128, 0, (0,), 128, True, True, 0, (37, 151)),
    (False, 3, 1, 1, 0, 128, 128, (256,), 256, True, True, 2, (20, 24)),
    (True, 5, 2, 2, 1, 256, 0, (), 128, True, False, 1, (30, 70)),
    (True, 3, 1, 1, 0, 128, 0, (), 128, True, False, 0, (19, 130)),
    (False, 3, 1, 1, 0, 96, 0, (96,), 128, False, False, 0, (8, 64)),
    (False, 3, 1, 1, 0, 256, 0, (256,), 256, True, True, 0, (6, 200)),  # GeoFF stage 3's 200-column grid
]


@pytest.mark.parametrize("case", RS_CASES, ids=[str(i) for i in range(len(RS_CASES))])
def test_wide_rolling_loop_bitwise(case, monkeypatch):
    from damvsnet_amd.frontend_hip import HipConv2d, planes
    tr, k, s, p, op, c0, c1, geo, cout, relu, pre, post_up, (H, W) = case
    g = torch.Generator().manual_seed(7)
    B = 2
    cin = c0 + c1 + len(geo)
    conv = (nn.ConvTranspose2d(cin, cout, k, stride=s, padding=p, output_padding=op) if tr
            else nn.Conv2d(cin, cout, k, stride=s, padding=p))
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.2)
        conv.bias.copy_(torch.randn(conv.bias.shape, generator=g) * 0.1)
    tensor_at = [c for c in range(cin) if c not in geo]
    at = dict(c0=c0, c0_at=tensor_at[0])
    if c1:
        at.update(c1=c1, c1_at=tensor_at[c0])
    L = HipConv2d(conv, torch.float32, relu, geo_at=geo, **at)
    a = torch.randn(B, H, W, c0, generator=g).to(DEV)
    b = torch.randn(B, H, W, c1, generator=g).to(DEV) if c1 else None
    gp = planes(torch.randn(B, len(geo), H, W, generator=g).to(DEV)) if geo else ()
    Ho, Wo = (H - 1) * s - 2 * p + k + op if tr else (H + 2 * p - k) // s + 1, \
        (W - 1) * s - 2 * p + k + op if tr else (W + 2 * p - k) // s + 1
    rp = torch.randn(B, Ho, Wo, L.cout_store, generator=g).to(DEV) if pre else None
    rq = torch.randn(B, Ho // post_up, Wo // post_up, L.cout_store, generator=g).to(DEV) if post_up else None
    run = lambda: L(B, H, W, a, b, geo=gp, res_pre=rp, res_post=rq, post_up=max(post_up, 1))  # noqa: E731
    monkeypatch.delenv("DAMVS_WIDE_RS", raising=False)
    y_rs = run()
    monkeypatch.setenv("DAMVS_WIDE_RS", "0")
    y_ag = run()
    torch.cuda.synchronize()
    assert torch.isfinite(y_rs).all()
    assert torch.equal(y_rs, y_ag)


# fp32 stride-2 128-channel wide layers on one-row q-tiles (the default, conv2d_wide_kernel R1) against the 2-row tiles
# (DAMVS_WIDE_S2R1=0): the same AG loop per accumulator, so bitwise equal. GeoBlock conv1 (two inputs + plane), 128+g -> 256, ragged.
S2R1_CASES = [
    (False, 3, 2, 1, 0, 128, 128, (256,), 256, True, False, 0, (37, 151)),
    (False, 3, 2, 1, 0, 128, 0, (128,), 256, True, False, 0, (20, 24)),
    (False, 3, 2, 1, 0, 64, 64, (0,), 128, False, True, 0, (30, 400)),
]


@pytest.mark.parametrize("case", S2R1_CASES, ids=[str(i) for i in range(len(S2R1_CASES))])
def test_wide_s2_one_row_tiles_bitwise(case, monkeypatch):
    from damvsnet_amd.frontend_hip import HipConv2d, planes
    tr, k, s, p, op, c0, c1, geo, cout, relu, pre, post_up, (H, W) = case
    g = torch.Generator().manual_seed(11)
    B = 2
    cin = c0 + c1 + len(geo)
    conv = nn.Conv2d(cin, cout, k, stride=s, padding=p)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.2)
        conv.bias.copy_(torch.randn(conv.bias.shape, generator=g) * 0.1)
    tensor_at = [c for c in range(cin) if c not in geo]
    at = dict(c0=c0, c0_at=tensor_at[0])
    if c1:
        at.update(c1=c1, c1_at=tensor_at[c0])
    L = HipConv2d(conv, torch.float32, relu, geo_at=geo, **at)
    a = torch.randn(B, H, W, c0, generator=g).to(DEV)
    b = torch.randn(B, H, W, c1, generator=g).to(DEV) if c1 else None
    gp = planes(torch.randn(B, len(geo), H, W, generator=g).to(DEV)) if geo else ()
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    rp = torch.randn(B, Ho, Wo, L.cout_store, generator=g).to(DEV) if pre else None
    run = lambda: L(B, H, W, a, b, geo=gp, res_pre=rp)  # noqa: E731
    monkeypatch.setenv("DAMVS_WIDE_S2R1", "0")
    y2 = run()
    monkeypatch.delenv("DAMVS_WIDE_S2R1")  # default: one-row tiles
    y1 = run()
    torch.cuda.synchronize()
    assert torch.isfinite(y2).all()
    assert torch.equal(y1, y2)


# fp32 layers on the 32-K gather kernel (conv2d_mfma_kernel K32: 8 channels per lane and K step, 16x16x32 split-f16
# MFMAs) against the 16-K form (DAMVS_CONV2D_G32=0): the same products summed in another order, so equal to fp32
# rounding. FeatureNet's k5 s2 convs, the 1x1 GeoBlock downsamples (two inputs + plane, stride 2), the FPN inner conv
# with the upsampled residual, GeoFF's full-resolution stride-2 conv with the depth plane.
G32_CASES = [
    (False, 5, 2, 2, 0, 8, 0, (), 16, True, False, 0, (60, 84)),
    (False, 5, 2, 2, 0, 16, 0, (), 32, True, False, 0, (30, 44)),
    (False, 1, 2, 0, 0, 128, 128, (256,), 256, True, False, 0, (20, 26)),
    (False, 1, 1, 0, 0, 64, 0, (64,), 128, True, False, 0, (19, 30)),
    (False, 1, 1, 0, 0, 16, 0, (), 32, False, False, 2, (24, 40)),
    (False, 3, 2, 1, 0, 8, 0, (8,), 16, True, False, 0, (40, 72)),
]


@pytest.mark.parametrize("case", G32_CASES, ids=[str(i) for i in range(len(G32_CASES))])
def test_gather_conv2d_k32_vs_k16_fp32(case, monkeypatch):
    from damvsnet_amd.frontend_hip import HipConv2d, planes
    tr, k, s, p, op, c0, c1, geo, cout, relu, pre, post_up, (H, W) = case
    g = torch.Generator().manual_seed(11)
    B = 2
    cin = c0 + c1 + len(geo)
    conv = nn.Conv2d(cin, cout, k, stride=s, padding=p)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.2)
        conv.bias.copy_(torch.randn(conv.bias.shape, generator=g) * 0.1)
    tensor_at = [c for c in range(cin) if c not in geo]
    at = dict(c0=c0, c0_at=tensor_at[0])
    if c1:
        at.update(c1=c1, c1_at=tensor_at[c0])
    L = HipConv2d(conv, torch.float32, relu, geo_at=geo, **at)
    a = torch.randn(B, H, W, c0, generator=g).to(DEV)
    b = torch.randn(B, H, W, c1, generator=g).to(DEV) if c1 else None
    gp = planes(torch.randn(B, len(geo), H, W, generator=g).to(DEV)) if geo else ()
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    rq = torch.randn(B, Ho // post_up, Wo // post_up, L.cout_store, generator=g).to(DEV) if post_up else None
    run = lambda: L(B, H, W, a, b, geo=gp, res_post=rq, post_up=max(post_up, 1))  # noqa: E731
    monkeypatch.delenv("DAMVS_CONV2D_G32", raising=False)
    y32 = run()
    monkeypatch.setenv("DAMVS_CONV2D_G32", "0")
    y16 = run()
    torch.cuda.synchronize()
    assert torch.isfinite(y32).all()
    assert rel_max(y32.cpu().numpy(), y16.cpu().numpy()) < 2e-6


# fp32 narrow layers on the halo kernel's rolling tap loop (conv2d_halo_kernel RS) against its plain W32 loop
# (DAMVS_HALO_RS=0): the same MFMA sequence per accumulator, so bitwise equal. One-slice layers with the plane (32+g ->
# 32 and -> 16), the k5 s2 transposed decoders (4 phases, 4 slices), two inputs, ragged tiles.
HALO_RS_CASES = [
    (False, 3, 1, 1, 0, 32, 0, (32,), 32, True, True, 0, (37, 151)),
    (False, 3, 1, 1, 0, 32, 0, (32,), 16, True, False, 0, (20, 70)),
    (True, 5, 2, 2, 1, 128, 0, (), 32, True, False, 1, (30, 70)),
    (True, 5, 2, 2, 1, 64, 0, (), 32, True, False, 1, (19, 40)),
    (False, 3, 1, 1, 0, 32, 32, (), 32, True, False, 0, (24, 66)),
]


@pytest.mark.parametrize("case", HALO_RS_CASES, ids=[str(i) for i in range(len(HALO_RS_CASES))])
def test_halo_rolling_loop_bitwise(case, monkeypatch):
    from damvsnet_amd.frontend_hip import HipConv2d, planes
    tr, k, s, p, op, c0, c1, geo, cout, relu, pre, post_up, (H, W) = case
    g = torch.Generator().manual_seed(5)
    B = 2
    cin = c0 + c1 + len(geo)
    conv = (nn.ConvTranspose2d(cin, cout, k, stride=s, padding=p, output_padding=op) if tr
            else nn.Conv2d(cin, cout, k, stride=s, padding=p))
    with torch.no_grad():
        conv.weight.copy_(torch.randn(conv.weight.shape, generator=g) * 0.2)
        conv.bias.copy_(torch.randn(conv.bias.shape, generator=g) * 0.1)
    tensor_at = [c for c in range(cin) if c not in geo]
    at = dict(c0=c0, c0_at=tensor_at[0])
    if c1:
        at.update(c1=c1, c1_at=tensor_at[c0])
    L = HipConv2d(conv, torch.float32, relu, geo_at=geo, **at)
    a = torch.randn(B, H, W, c0, generator=g).to(DEV)
    b = torch.randn(B, H, W, c1, generator=g).to(DEV) if c1 else None
    gp = planes(torch.randn(B, len(geo), H, W, generator=g).to(DEV)) if geo else ()
    Ho, Wo = ((H - 1) * s - 2 * p + k + op, (W - 1) * s - 2 * p + k + op) if tr else \
        ((H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1)
    rp = torch.randn(B, Ho, Wo, L.cout_store, generator=g).to(DEV) if pre else None
    rq = torch.randn(B, Ho // post_up, Wo // post_up, L.cout_store, generator=g).to(DEV) if post_up else None
    run = lambda: L(B, H, W, a, b, geo=gp, res_pre=rp, res_post=rq, post_up=max(post_up, 1))  # noqa: E731
    monkeypatch.delenv("DAMVS_HALO_RS", raising=False)
    y_rs = run()
    monkeypatch.setenv("DAMVS_HALO_RS", "0")
    y_pl = run()
    torch.cuda.synchronize()
    assert torch.isfinite(y_rs).all()
    assert torch.equal(y_rs, y_pl)
