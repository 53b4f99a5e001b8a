"""ORACLE — test infrastructure only. NOT part of the product.

A CPU restatement (PyTorch CPU ops, NCDHW, float32 unless asked otherwise) of the
reference's cascade-MVS forward (wsmtht520/DAMVSNet, models/cas_mvsnet.py). Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it,
and only as the checker / the CPU baseline; the product path (``damvsnet_amd``) never
imports or calls it and fails loudly when its HIP library is missing.

Parity pinning: the reference has no tests or fixtures of its own, so
this restatement is pinned against golden vectors produced by importing the reference in
the build container (``tests/golden/make_golden.py``, outputs committed under
``tests/golden/``) plus the analytic known-answer tests of SURVEY.md section 4.

Every function is functional over a flat ``state_dict`` (the reference's keys) and cites
the reference lines it restates.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

EPS = 1e-12  # models/module.py:10
BN_EPS = 1e-5  # nn.BatchNorm defaults used by every BN in the reference


# --------------------------------------------------------------------------- helpers

def _bn(x, sd, p):
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"], sd[p + ".bias"],
                        training=False, eps=BN_EPS)


def compose_proj(P):
    """[K @ E[:3,:4]; E[3,:]] for a (B,2,4,4) projection pair — models/cas_mvsnet.py:44-47."""
    out = P[:, 0].clone()
    out[:, :3, :4] = torch.matmul(P[:, 1, :3, :3], P[:, 0, :3, :4])
    return out


# --------------------------------------------------------------------------- warp (A3)

def bilinear_zeros(src, ix, iy):
    """Bilinear sampling with zero padding at pixel coords (ix, iy) — the arithmetic of
    F.grid_sample(mode='bilinear', padding_mode='zeros') used at models/module.py:328-329.

    src (B,C,H,W); ix, iy (B,P) -> (B,C,P). Corner weights and accumulation order nw, ne, sw, se.
    """
    B, C, H, W = src.shape
    x0 = torch.floor(ix)
    y0 = torch.floor(iy)
    x1, y1 = x0 + 1, y0 + 1
    taps = ((x0, y0, (x1 - ix) * (y1 - iy)), (x1, y0, (ix - x0) * (y1 - iy)),
            (x0, y1, (x1 - ix) * (iy - y0)), (x1, y1, (ix - x0) * (iy - y0)))
    flat = src.reshape(B, C, H * W)
    out = torch.zeros(B, C, ix.shape[1], dtype=src.dtype)
    for tx, ty, wgt in taps:
        valid = (tx >= 0) & (tx <= W - 1) & (ty >= 0) & (ty <= H - 1)
        idx = (ty.clamp(0, H - 1) * W + tx.clamp(0, W - 1)).long()
        val = torch.gather(flat, 2, idx.unsqueeze(1).expand(B, C, idx.shape[1]))
        out = out + val * (wgt * valid.to(src.dtype)).unsqueeze(1)
    return out


def homo_warping(src_fea, src_proj, ref_proj, depth_values, impl="grid_sample"):
    """models/module.py:297-332.

    Grid normalised with (W-1)/2 (align-corners style, :323-324) but sampled at
    grid_sample's default align_corners=False (:328): effective source pixel
    ix = ((u/((W-1)/2) - 1 + 1) * W - 1) / 2, zero outside.
    ``impl='gather'`` is an explicit restatement of the sampler; ``'grid_sample'`` calls the
    same PyTorch op the reference calls (used for the CPU baseline's speed).
    """
    B, C, H, W = src_fea.shape
    D = depth_values.shape[1]
    dt = src_fea.dtype
    proj = torch.matmul(src_proj.to(dt), torch.inverse(ref_proj.to(dt)))
    rot, trans = proj[:, :3, :3], proj[:, :3, 3:4]
    y, x = torch.meshgrid(torch.arange(H, dtype=dt), torch.arange(W, dtype=dt), indexing="ij")
    xyz = torch.stack((x.reshape(-1), y.reshape(-1), torch.ones(H * W, dtype=dt))).unsqueeze(0).repeat(B, 1, 1)
    rot_xyz = torch.matmul(rot, xyz)
    p = rot_xyz.unsqueeze(2) * depth_values.to(dt).reshape(B, 1, D, -1) + trans.reshape(B, 3, 1, 1)
    px = p[:, 0] / p[:, 2]
    py = p[:, 1] / p[:, 2]
    gx = px / ((W - 1) / 2) - 1
    gy = py / ((H - 1) / 2) - 1
    if impl == "grid_sample":
        grid = torch.stack((gx, gy), dim=3).reshape(B, D * H, W, 2)
        out = F.grid_sample(src_fea, grid, mode="bilinear", padding_mode="zeros", align_corners=False)
        return out.reshape(B, C, D, H, W)
    ix = ((gx + 1) * W - 1) / 2
    iy = ((gy + 1) * H - 1) / 2
    return bilinear_zeros(src_fea, ix.reshape(B, -1), iy.reshape(B, -1)).reshape(B, C, D, H, W)


# --------------------------------------------------------------------------- aggregation (A4, A4v, A5)

def agg_weight(x, sd, p):
    """AggWeightNetVolume.forward — models/module.py:544-563 (conv0 unused, :561)."""
    w = F.relu(_bn(F.conv3d(x, sd[p + ".w_net.0.conv.weight"]), sd, p + ".w_net.0.bn"))
    return F.relu(_bn(F.conv3d(w, sd[p + ".w_net.1.conv.weight"]), sd, p + ".w_net.1.bn"))


def aggregate(features, proj, hyps, sd, stage_idx, mode="adaptive", warp_impl="grid_sample"):
    """Cost-volume construction of DepthNet.forward — models/cas_mvsnet.py:26-87."""
    N = len(features)
    D = hyps.shape[1]
    ref, srcs = features[0], features[1:]
    ref_vol = ref.unsqueeze(2).repeat(1, 1, D, 1, 1)
    refP = compose_proj(proj[:, 0])
    if mode == "variance":
        vsum, vsq = ref_vol, ref_vol ** 2
    acc = None
    for v, src in enumerate(srcs, start=1):
        warped = homo_warping(src, compose_proj(proj[:, v]), refP, hyps, impl=warp_impl)
        if mode == "variance":
            vsum = vsum + warped
            vsq = vsq + warped ** 2
        else:
            x = (ref_vol - warped).pow_(2)
            w = agg_weight(x, sd, "DepthNet.weight_net.%d" % stage_idx)
            acc = (w + 1) * x if acc is None else acc + (w + 1) * x
    if mode == "variance":
        return vsq.div_(N).sub_(vsum.div_(N).pow_(2))
    return acc / (N - 1)


# --------------------------------------------------------------------------- CostRegNet (A6)

def costregnet(x, sd, p):
    """CostRegNet.forward — models/module.py:510-541 (Conv3d/Deconv3d wrappers :117-202)."""
    def conv(t, name, stride=1):
        return F.relu(_bn(F.conv3d(t, sd[p + "." + name + ".conv.weight"], stride=stride, padding=1), sd,
                          p + "." + name + ".bn"))

    def deconv(t, name):
        y = F.conv_transpose3d(t, sd[p + "." + name + ".conv.weight"], stride=2, padding=1, output_padding=1)
        return F.relu(_bn(y, sd, p + "." + name + ".bn"))

    c0 = conv(x, "conv0")
    c2 = conv(conv(c0, "conv1", 2), "conv2")
    c4 = conv(conv(c2, "conv3", 2), "conv4")
    y = conv(conv(c4, "conv5", 2), "conv6")
    y = c4 + deconv(y, "conv7")
    y = c2 + deconv(y, "conv9")
    y = c0 + deconv(y, "conv11")
    return F.conv3d(y, sd[p + ".prob.weight"], padding=1)


# --------------------------------------------------------------------------- regression (A7, A8, A9)

def regression(logits, hyps, prob_volume_init=None):
    """Softmax, depth, photometric confidence, exp-variance — models/cas_mvsnet.py:105-124."""
    pre = logits.squeeze(1) if logits.dim() == 5 else logits
    if prob_volume_init is not None:
        pre = pre + prob_volume_init
    D = pre.shape[1]
    prob = F.softmax(pre, dim=1)
    depth = torch.sum(prob * hyps, 1)  # depth_regression, models/module.py:609-615
    sum4 = 4 * F.avg_pool3d(F.pad(prob.unsqueeze(1), pad=(0, 0, 0, 0, 1, 2)), (4, 1, 1), stride=1, padding=0).squeeze(1)
    idx = torch.sum(prob * torch.arange(D, dtype=prob.dtype).view(1, D, 1, 1), 1).long().clamp(0, D - 1)
    conf = torch.gather(sum4, 1, idx.unsqueeze(1)).squeeze(1)
    var = 3 * torch.sum((hyps - depth.unsqueeze(1)) ** 2 * prob, dim=1) ** 0.5
    return {"depth": depth, "photometric_confidence": conf, "variance": var, "prob_volume": prob,
            "depth_values": hyps}


def depthnet_stage(stage_idx, features, proj, hyps, sd, mode="adaptive", share_cr=False, warp_impl="grid_sample",
                   prob_volume_init=None):
    """DepthNet.forward — models/cas_mvsnet.py:18-134."""
    vol = aggregate(features, proj, hyps, sd, stage_idx, mode, warp_impl)
    cr = "cost_regularization" if share_cr else "cost_regularization.%d" % stage_idx
    logits = costregnet(vol, sd, cr)
    return regression(logits, hyps, prob_volume_init)


# --------------------------------------------------------------------------- sampling glue (A10)

def bilinear_resize(x, size):
    """F.interpolate(mode='bilinear', align_corners=False) as used at models/cas_mvsnet.py:250-253."""
    return F.interpolate(x, size, mode="bilinear", align_corners=False)


def uncertainty_aware_samples(cur_depth, exp_var, ndepth, shape):
    """models/module.py:999-1038. cur_depth (B,Dv) at stage 1, else (B,1,H,W) with exp_var."""
    B, H, W = shape
    if cur_depth.dim() == 2:
        dmin, dmax = cur_depth[:, 0], cur_depth[:, -1]
        itv = (dmax - dmin) / (ndepth - 1)
        s = dmin.unsqueeze(1) + torch.arange(0, ndepth, dtype=cur_depth.dtype).reshape(1, -1) * itv.unsqueeze(1)
        return s.unsqueeze(-1).unsqueeze(-1).repeat(1, 1, H, W)
    low = -torch.min(cur_depth, exp_var)
    high = exp_var
    step = (high - low) / (float(ndepth) - 1)
    offs = [3 * (low + step * i) / (exp_var + EPS) for i in range(ndepth)]
    samps = [cur_depth + low + step * i + EPS for i in range(ndepth)]
    return torch.cat(samps, 1) + F.softmax(torch.cat(offs, 1), dim=1) * step


def stage_hypotheses(stage_idx, depth_values, prev_depth, prev_var, ndepth, H, W, scale):
    """Hypotheses handed to DepthNet at one stage — models/cas_mvsnet.py:238-296."""
    B = depth_values.shape[0]
    if prev_depth is None:
        cur, var = depth_values, None
    else:
        cur = bilinear_resize(prev_depth.unsqueeze(1), [H, W])
        var = bilinear_resize(prev_var.unsqueeze(1), [H, W])
    full = uncertainty_aware_samples(cur, var, ndepth, (B, H, W))
    return F.interpolate(full.unsqueeze(1), [ndepth, H // scale, W // scale], mode="trilinear",
                         align_corners=False).squeeze(1)


# --------------------------------------------------------------------------- 2D front-end (f1)

def _cbr2(x, sd, p, stride=1, padding=0, relu=True):
    y = _bn(F.conv2d(x, sd[p + ".conv.weight"], stride=stride, padding=padding), sd, p + ".bn")
    return F.relu(y) if relu else y


def feature_net(x, sd, arch_mode="fpn", p="feature"):
    """FeatureNet.forward — models/module.py:417-462 (fpn) and unet branch."""
    c0 = _cbr2(_cbr2(x, sd, p + ".conv0.0", 1, 1), sd, p + ".conv0.1", 1, 1)
    c1 = _cbr2(c0, sd, p + ".conv1.0", 2, 2)
    c1 = _cbr2(_cbr2(c1, sd, p + ".conv1.1", 1, 1), sd, p + ".conv1.2", 1, 1)
    c2 = _cbr2(c1, sd, p + ".conv2.0", 2, 2)
    c2 = _cbr2(_cbr2(c2, sd, p + ".conv2.1", 1, 1), sd, p + ".conv2.2", 1, 1)
    out = {"stage1": F.conv2d(c2, sd[p + ".out1.weight"])}
    if arch_mode == "fpn":
        f = F.interpolate(c2, scale_factor=2, mode="nearest") + F.conv2d(c1, sd[p + ".inner1.weight"], sd[p + ".inner1.bias"])
        out["stage2"] = F.conv2d(f, sd[p + ".out2.weight"], padding=1)
        f = F.interpolate(f, scale_factor=2, mode="nearest") + F.conv2d(c0, sd[p + ".inner2.weight"], sd[p + ".inner2.bias"])
        out["stage3"] = F.conv2d(f, sd[p + ".out3.weight"], padding=1)
        return out

    def fuse(skip, t, q):
        y = F.conv_transpose2d(t, sd[q + ".deconv.conv.weight"], stride=2, padding=1, output_padding=1)
        y = y[:, :, :2 * t.shape[2], :2 * t.shape[3]]
        y = F.relu(_bn(y, sd, q + ".deconv.bn"))
        return _cbr2(torch.cat((y, skip), 1), sd, q + ".conv", 1, 1)

    f = fuse(c1, c2, p + ".deconv1")
    out["stage2"] = F.conv2d(f, sd[p + ".out2.weight"])
    out["stage3"] = F.conv2d(fuse(c0, f, p + ".deconv2"), sd[p + ".out3.weight"])
    return out


def _seq_cbr(x, sd, p, stride, padding):
    return F.relu(_bn(F.conv2d(x, sd[p + ".0.weight"], stride=stride, padding=padding), sd, p + ".1"))


def _seq_dbr(x, sd, p, stride, padding, output_padding):
    y = F.conv_transpose2d(x, sd[p + ".0.weight"], stride=stride, padding=padding, output_padding=output_padding)
    return F.relu(_bn(y, sd, p + ".1"))


def _geo_block(x, g1, g2, sd, p, stride):
    """BasicBlockGeo.forward — models/geometry.py:410-433."""
    xg = torch.cat((x, g1), 1)
    y = F.relu(_bn(F.conv2d(xg, sd[p + ".conv1.weight"], stride=stride, padding=1), sd, p + ".bn1"))
    y = _bn(F.conv2d(torch.cat((g2, y), 1), sd[p + ".conv2.weight"], padding=1), sd, p + ".bn2")
    if (p + ".downsample.0.weight") in sd:
        idt = _bn(F.conv2d(xg, sd[p + ".downsample.0.weight"], stride=stride), sd, p + ".downsample.1")
    else:
        idt = x
    return F.relu(y + idt)


def _sparse_pool(d, m):
    """SparseDownSampleClose(stride=2) — models/geometry.py:443-455."""
    enc = -(1 - m) * 600 - d
    dd = -F.max_pool2d(enc, 2, 2)
    mm = F.max_pool2d(m, 2, 2)
    return dd - (1 - mm) * 600, mm


def geo_feature_fusion(rgb, depth, confidence, depth_values, stage_idx, origin_feat, sd, p="GeoFeatureFusionNet"):
    """GeoFeatureFusion.forward, 'z' encoding / 'basic' mask — models/geometry.py:87-277."""
    dmin = depth_values[:, 0, None, None, None]
    dmax = depth_values[:, -1, None, None, None]
    d = (depth - dmin) / (dmax - dmin)
    vm = torch.where(d > 0, torch.ones_like(d), torch.zeros_like(d))
    d2, m2 = _sparse_pool(d, vm)
    d3, m3 = _sparse_pool(d2, m2)
    d4, _ = _sparse_pool(d3, m3)
    q = p + "."
    r0 = _seq_cbr(torch.cat((rgb, d), 1), sd, q + "rgb_conv_init", 1, 2)
    r1 = _geo_block(r0, d, d2, sd, q + "rgb_encoder_layer1", 2)
    r2 = _geo_block(r1, d2, d2, sd, q + "rgb_encoder_layer2", 1)
    r3 = _geo_block(r2, d2, d3, sd, q + "rgb_encoder_layer3", 2)
    r4 = _geo_block(r3, d3, d3, sd, q + "rgb_encoder_layer4", 1)
    r5 = _geo_block(r4, d3, d4, sd, q + "rgb_encoder_layer5", 2)
    r4p = _seq_dbr(r5, sd, q + "rgb_decoder_layer4", 2, 2, 1) + r4
    r2p = _seq_dbr(r4p, sd, q + "rgb_decoder_layer2", 2, 2, 1) + r2
    r0p = _seq_dbr(r2p, sd, q + "rgb_decoder_layer0", 1, 1, 0) + r1
    rp = _seq_dbr(r0p, sd, q + "rgb_decoder_layer", 2, 2, 1) + r0
    rgb_out = _seq_dbr(rp, sd, q + "rgb_decoder_output", 1, 1, 0)
    s0 = _seq_cbr(torch.cat((d, rgb_out[:, 0:1]), 1), sd, q + "depth_conv_init", 1, 2)
    s1 = _geo_block(s0, d, d2, sd, q + "depth_layer1", 2)
    s2 = _geo_block(s1, d2, d2, sd, q + "depth_layer2", 1)
    s3 = _geo_block(torch.cat([r2p, s2], 1), d2, d3, sd, q + "depth_layer3", 2)
    s4 = _geo_block(s3, d3, d3, sd, q + "depth_layer4", 1)
    s5 = _geo_block(torch.cat([r4p, s4], 1), d3, d4, sd, q + "depth_layer5", 2)
    dec3 = _seq_dbr(r5 + s5, sd, q + "decoder_layer3", 2, 2, 1)
    dec4 = _seq_dbr(s4 + dec3, sd, q + "decoder_layer4", 1, 1, 0)
    dec5 = _seq_dbr(dec4, sd, q + "decoder_layer5", 2, 2, 1)
    dec6 = _seq_dbr(dec5, sd, q + "decoder_layer6", 1, 1, 0)
    if stage_idx == 1:
        f = _seq_dbr(s1 + dec6, sd, q + "rgbdepth_decoder_stage2", 2, 2, 1)
        return _seq_dbr(f + origin_feat, sd, q + "final_decoder_stage2", 1, 1, 0)
    dec7 = _seq_dbr(dec6, sd, q + "decoder_layer7", 2, 2, 1)
    f = _seq_dbr(s0 + dec7, sd, q + "rgbdepth_decoder_stage3", 1, 1, 0)
    return _seq_dbr(f + origin_feat, sd, q + "final_decoder_stage3", 1, 1, 0)


# --------------------------------------------------------------------------- full forward (A11)

STAGE_SCALE = (4, 2, 1)  # models/cas_mvsnet.py:154-164


def cascade_forward(sd, imgs, proj_matrices, depth_values, ndepths=(48, 32, 8), agg_mode="adaptive",
                    share_cr=False, arch_mode="fpn", warp_impl="grid_sample", stage_hook=None, depthnet=None):
    """CascadeMVSNet.forward — models/cas_mvsnet.py:190-319 (inference, grad_method 'detach').

    ``stage_hook(name)`` (optional) is called around the major phases for timing. ``depthnet`` (optional, tests
    only) replaces depthnet_stage: called as depthnet(stage_idx, features, proj, hyps) -> the stage's output dict
    (e.g. a depth-sharded stage, tests/test_sharded.py).
    Returns the reference's output dict: per-stage dicts plus stage-3 keys at top level.
    """
    hook = stage_hook or (lambda name: None)
    B, N, _, H, W = imgs.shape
    hook("features")
    feats = [feature_net(imgs[:, v], sd, arch_mode) for v in range(N)]
    outputs = {}
    depth = var = conf = None
    for s, nd in enumerate(ndepths):
        name = "stage%d" % (s + 1)
        fs = [f[name] for f in feats]
        if s >= 1:
            hook(name + ".geofusion")
            rgb = F.interpolate(imgs[:, 0], scale_factor=1.0 / 2 ** (2 - s), mode="bilinear", align_corners=False)
            dl = F.interpolate(depth.unsqueeze(1), scale_factor=2, mode="bilinear", align_corners=False)
            cl = F.interpolate(conf.unsqueeze(1), scale_factor=2, mode="bilinear", align_corners=False)
            fs[0] = geo_feature_fusion(rgb, dl, cl, depth_values, s, fs[0], sd)
        hook(name + ".hypotheses")
        hyps = stage_hypotheses(s, depth_values, depth, var, nd, H, W, STAGE_SCALE[s])
        hook(name + ".depthnet")
        if depthnet is not None:
            out = depthnet(s, fs, proj_matrices[name], hyps)
        else:
            out = depthnet_stage(s, fs, proj_matrices[name], hyps, sd, agg_mode, share_cr, warp_impl)
        depth, conf, var = out["depth"], out["photometric_confidence"], out["variance"]
        outputs[name] = out
        outputs.update(out)
    hook("end")
    return outputs
