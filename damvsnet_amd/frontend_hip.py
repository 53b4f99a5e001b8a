"""The 2D front-end on libdamvs: FeatureNet and GeoFeatureFusion
as chains of fused HIP conv2d layers (damvs_conv2d_*), NHWC end to end.

Each reference op sequence maps to one launch: conv + BN + ReLU (+ the residual add that follows,
before or after the ReLU), with the reference's torch.cat of feature maps and 1-channel depth
planes folded into the conv's inputs. Weights come from the BN-folded copies
(``frontend_fold.fold_frontend``); the reference-keyed modules stay the parameter owners.

Reference forwards mirrored: FeatureNet.forward models/module.py:417-462 (fpn and unet),
GeoFeatureFusion.forward models/geometry.py:87-277, BasicBlockGeo.forward geometry.py:410-433,
SparseDownSampleClose geometry.py:443-455.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch
import torch.nn as nn

from . import _capi
from ._capi import check, ptr
from .engine import DTYPES
from .frontend import ConvBNReLU2d, DeconvBNReLU2d, GeoBlock


class HipConv2d:
    """One fused conv2d / conv-transpose2d layer resident on the GPU (damvs_conv2d handle)."""

    def __init__(self, conv, dtype, relu, c0=0, c0_at=0, c1=0, c1_at=0, geo_at=()):
        lib = _capi.load_library()
        self._lib = lib
        tr = isinstance(conv, nn.ConvTranspose2d)
        w = conv.weight.detach().to("cpu", torch.float32).contiguous()
        b = conv.bias.detach().to("cpu", torch.float32).contiguous() if conv.bias is not None else None
        cin = w.shape[0] if tr else w.shape[1]
        cout = w.shape[1] if tr else w.shape[0]
        d = _capi.DamvsConv2dDesc()
        d.transposed = int(tr)
        d.kernel, d.stride, d.padding = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        d.output_padding = conv.output_padding[0] if tr else 0
        d.cin, d.cout = cin, cout
        d.c0, d.c0_at, d.c1, d.c1_at = c0, c0_at, c1, c1_at
        d.ngeo = len(geo_at)
        for i, g in enumerate(geo_at):
            d.geo_at[i] = g
        d.relu = int(relu)
        h = ctypes.c_void_p()
        check(lib.damvs_conv2d_create(ctypes.byref(d), ptr(w), ptr(b), DTYPES[dtype], ctypes.byref(h)))
        self.handle, self.dtype, self.ngeo = h, dtype, len(geo_at)
        self.desc = "%s k%d s%d" % ("convT" if tr else "conv", d.kernel, d.stride)
        self.kernel, self.stride, self.transposed = d.kernel, d.stride, tr
        self.cout = cout
        self.cout_store = (cout + 3) // 4 * 4

    def __del__(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            try:
                self._lib.damvs_conv2d_destroy(self.handle)
            except Exception:
                pass

    def out_shape(self, B, Hi, Wi):
        ho, wo, cs = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(self._lib.damvs_conv2d_out_size(self.handle, Hi, Wi, ctypes.byref(ho), ctypes.byref(wo),
                                              ctypes.byref(cs)))
        return (B, ho.value, wo.value, cs.value)

    def __call__(self, B, Hi, Wi, in0=None, in1=None, geo=(), res_pre=None, res_post=None, post_up=1, out=None):
        dev = (in0 if in0 is not None else geo[0][0]).device
        shape = self.out_shape(B, Hi, Wi)
        if out is None:
            out = torch.empty(shape, device=dev, dtype=self.dtype)
        elif tuple(out.shape) != shape or out.dtype != self.dtype or not out.is_contiguous():
            raise ValueError("conv2d out: need a contiguous %s %s tensor, got %s %s"
                             % (self.dtype, shape, out.dtype, tuple(out.shape)))
        gp = gs = None
        if self.ngeo:
            assert len(geo) == self.ngeo, (len(geo), self.ngeo)
            gp = (ctypes.c_void_p * 4)(*([g.data_ptr() for g, _ in geo] + [0] * (4 - len(geo))))
            gs = (ctypes.c_longlong * 4)(*([st for _, st in geo] + [0] * (4 - len(geo))))
        check(self._lib.damvs_conv2d_forward(self.handle, _capi.stream_ptr(dev), B, Hi, Wi, ptr(in0), ptr(in1), gp,
                                             gs, ptr(res_pre), ptr(res_post), post_up, ptr(out)))
        return out


def planes(t):
    """(B, C, H, W) fp32 tensor -> list of C (plane view, batch stride) for the geo inputs. Rows must be
    dense (a view of a larger tensor such as imgs[:, v] is taken as is, its batch stride passed along)."""
    t = t.float()
    if t.stride(3) != 1 or t.stride(2) != t.shape[3] or t.stride(1) != t.shape[2] * t.shape[3]:
        t = t.contiguous()
    return [(t[:, c], t.stride(0)) for c in range(t.shape[1])]


def sparse_depth_pyramid(depth, depth_values, mask=None):
    """GeoFeatureFusion's normalised depth and its three SparseDownSampleClose levels
    (models/geometry.py:90-96, 117-119, 443-455) in three launches: depth (B,1,h,w) fp32 ->
    [d, d_s2, d_s3, d_s4] as (B,1,h>>l,w>>l) fp32. mask: the 'mean' valid mask (None: 'basic', d > 0)."""
    depth = depth.float().contiguous()
    B, _, h, w = depth.shape
    dv = depth_values.float().contiguous()
    mk = mask.float().contiguous() if mask is not None else None
    outs = [torch.empty(B, 1, h >> l, w >> l, device=depth.device) for l in range(4)]
    scratch = torch.empty(B * (h // 2) * (w // 2) + B * (h // 4) * (w // 4) + 1, device=depth.device)
    lib = _capi.load_library()
    check(lib.damvs_sparse_depth_pyramid(_capi.stream_ptr(depth.device), B, h, w, ptr(depth), ptr(dv), dv.shape[1],
                                         ptr(mk), *[ptr(o) for o in outs], ptr(scratch)))
    return outs


def fpn_top_layers(inner2, out3, dtype):
    """FeatureNet's last FPN level, out3(up2(f) + inner2(c0)) (models/module.py:455-459: nearest x2
    upsample, 1x1 conv with bias, 3x3 conv without bias, no BN/ReLU), re-associated so the
    32-channel full-resolution sum is never written:

      out3(up2(f))        = ConvTranspose2d(k4, s2, p1) of f whose taps are sums of out3's taps
                            (per axis, transposed tap a in {0..3} collects 3x3 taps S(a) =
                            {2}, {1,2}, {0,1}, {0}: nearest upsampling merges them pairwise);
      out3(inner2(c0))    = 3x3 conv of c0 with weights out3 . inner2 (8 -> 8);
      out3(inner2's bias) = the full 9-tap sum out3 . bias as that conv's bias, minus the taps that
                            fall outside the image at border pixels (zero padding of the sum):
                            damvs_conv2d_border_bias with corr[tap] = out3[tap] . bias.

    Returns (transposed layer on f, 3x3 layer on c0, corr [9 * cout] fp32, (Wt, Wc, bias) fp32 for the
    fused launch) — the second layer takes the first's output as its pre-activation residual."""
    W3 = out3.weight.detach().to("cpu", torch.float64)                 # (co, m, 3, 3)
    W1 = inner2.weight.detach().to("cpu", torch.float64)[:, :, 0, 0]   # (m, ci)
    b1 = inner2.bias.detach().to("cpu", torch.float64)                 # (m,)
    co, m = W3.shape[:2]
    ci = W1.shape[1]
    S = ((2,), (1, 2), (0, 1), (0,))
    wt = torch.zeros(m, co, 4, 4, dtype=torch.float64)
    for a in range(4):
        for b in range(4):
            wt[:, :, a, b] = sum(W3[:, :, ky, kx] for ky in S[a] for kx in S[b]).t()
    up = nn.ConvTranspose2d(m, co, 4, stride=2, padding=1, bias=False)
    up.weight.data = wt.float()
    corr = torch.einsum("omyx,m->yxo", W3, b1)                        # (3, 3, co)
    c0 = nn.Conv2d(ci, co, 3, padding=1, bias=True)
    c0.weight.data = torch.einsum("omyx,mi->oiyx", W3, W1).float()
    c0.bias.data = corr.sum((0, 1)).float()
    return (HipConv2d(up, dtype, False, c0=m), HipConv2d(c0, dtype, False, c0=ci), corr.reshape(-1).float().contiguous(),
            (up.weight.data.clone(), c0.weight.data.clone(), c0.bias.data.clone()))


def pack_fpn_top_split(wt, wc):
    """damvs_fpn_top_forward_f32's A chunks: pack_fpn_top's 15 x 64 x 8 values in fp32, scaled by 2^k (largest |A| in
    (2^13, 2^14]) and split into f16 halves hi = f16(v), lo = f16(v - hi); laid out [chunk][hi / lo][64 lanes][8].
    Returns (int16 view of the halves, wscale = 2^-k)."""
    A = _fpn_top_A(wt, wc)
    mx = float(A.abs().max())
    k = 0 if mx == 0.0 else 14 - math.frexp(mx)[1]
    v = A * (2.0 ** k)
    hi = v.half()
    lo = (v - hi.float()).half()
    return torch.stack([hi, lo], 1).contiguous().view(torch.int16), 2.0 ** -k


def _fpn_top_A(wt, wc):
    A = torch.zeros(15, 64, 8, dtype=torch.float32)
    for lane in range(64):
        g, row = lane >> 4, lane & 15
        px, co = row >> 3, row & 7
        for dy in range(3):
            kx = g - px
            if 0 <= kx <= 2:
                A[dy, lane] = wc[co, :, dy, kx]
        for py in range(2):
            for r2 in range(2):
                ky = py + 3 - 2 * (r2 + py)
                for xx in range(3):
                    kx = px + 3 - 2 * xx
                    if 0 <= kx <= 3:
                        A[3 + py * 6 + r2 * 3 + xx, lane] = wt[8 * g:8 * g + 8, co, ky, kx]
    return A


def pack_fpn_top(wt, wc):
    """MFMA A chunks of damvs_fpn_top_forward (15 x 64 lanes x 8 bf16): lane (g = lane >> 4, row = lane & 15)
    holds A[row][8g .. 8g+7], row = (output x parity px = row >> 3, channel co = row & 7).
      chunks 0-2  (3x3 conv, kernel row dy): k = (x-pair tap g: c0 column 2q-1+g, channel) -> Wc[co][ci][dy][g-px];
      chunks 3-14 (ConvTranspose k4 s2 p1, row parity py, input row m-1+rr with rr = r2+py, column q-1+xx):
                  k = channel 8g+e -> Wt[ci][co][ky][kx], ky = py+3-2rr, kx = px+3-2xx (zero outside 0..3).
    wt: (32, 8, 4, 4), wc: (8, 8, 3, 3) fp32."""
    return _fpn_top_A(wt, wc).to(torch.bfloat16)


class HipFeatureNet:
    """FeatureNet (fpn or unet) on libdamvs. Input imgs (B, 3, H, W) fp32; outputs NHWC."""

    def __init__(self, fnet, dtype):
        self.arch, self.num_stage = fnet.arch_mode, fnet.num_stage
        L = lambda m, relu, **k: HipConv2d(m, dtype, relu, **k)
        c00, c01 = fnet.conv0[0], fnet.conv0[1]
        self.c0 = [L(c00.conv, True, geo_at=(0, 1, 2)), L(c01.conv, True, c0=c01.conv.in_channels)]
        self.c1 = [L(m.conv, True, c0=m.conv.in_channels) for m in fnet.conv1]
        self.c2 = [L(m.conv, True, c0=m.conv.in_channels) for m in fnet.conv2]
        self.out1 = L(fnet.out1, False, c0=fnet.out1.in_channels)
        if self.arch == "fpn":
            self.inner1 = L(fnet.inner1, False, c0=fnet.inner1.in_channels)
            self.out2 = L(fnet.out2, False, c0=fnet.out2.in_channels)
            if self.num_stage == 3:
                self.top_up, self.top_c0, self.top_corr, (wt, wc, bc) = fpn_top_layers(fnet.inner2, fnet.out3, dtype)
                # one fused launch (damvs_fpn_top_forward, fp32: _f32 on split-f16 MFMAs); DAMVS_FPN_TOP_FUSED=0
                # keeps the two layers
                self.top_fused = None
                if wt.shape[0] == 32 and wt.shape[1] == 8 and wc.shape[1] == 8 and \
                        os.environ.get("DAMVS_FPN_TOP_FUSED", "1") != "0":
                    if dtype == torch.bfloat16:
                        self.top_fused = (pack_fpn_top(wt, wc), bc.float(), None)
                    elif dtype == torch.float32:
                        ap, ws = pack_fpn_top_split(wt, wc)
                        self.top_fused = (ap, bc.float(), ws)
        else:
            self.up = []
            for fu in [fnet.deconv1] + ([fnet.deconv2] if self.num_stage == 3 else []):
                co = fu.deconv.conv.out_channels
                self.up.append((L(fu.deconv.conv, True, c0=fu.deconv.conv.in_channels),
                                L(fu.conv.conv, True, c0=co, c0_at=0, c1=co, c1_at=co)))
            self.out2 = L(fnet.out2, False, c0=fnet.out2.in_channels)
            if self.num_stage == 3:
                self.out3 = L(fnet.out3, False, c0=fnet.out3.in_channels)

    # the kernels' 32-bit buffer offsets keep every operand below 2 GiB; the widest FeatureNet tensors are the
    # full-resolution 8-channel ones, so view groups are sized to keep those under this bound
    MAX_ACT_BYTES = 3 << 29  # 1.5 GiB

    def __call__(self, x):
        """x: (B, 3, H, W), or (B, N, 3, H, W) views batched view-major (row v*B + b) with no copy of the
        images: the first layer reads each view's planes in place, one launch per view. Views run in groups when one
        batch of all of them would pass the 32-bit offset bound (cfgE's 11 views x B=4 at 1920 x 1056 in fp32: 2.85 GB per
        8-channel activation); the groups' outputs are concatenated in view order."""
        if x.dim() == 5:
            Bv, N, _, H, W = x.shape
            es = torch.tensor([], dtype=self.c0[0].dtype).element_size()
            per_view = Bv * H * W * 8 * es
            if N > 1 and N * per_view > self.MAX_ACT_BYTES:
                g = max(1, self.MAX_ACT_BYTES // per_view)
                parts = [self(x[:, v:v + g]) for v in range(0, N, g)]
                return {k: torch.cat([p[k] for p in parts], 0) for k in parts[0]}
            B = N * Bv
            L = self.c0[0]
            t = torch.empty(L.out_shape(B, H, W), device=x.device, dtype=L.dtype)
            for v in range(N):
                L(Bv, H, W, geo=planes(x[:, v]), out=t[v * Bv:(v + 1) * Bv])
        else:
            B, _, H, W = x.shape
            t = self.c0[0](B, H, W, geo=planes(x))
        c0 = self.c0[1](B, H, W, t)
        h, w = c0.shape[1:3]
        t = c0
        for L in self.c1:
            t = L(B, t.shape[1], t.shape[2], t)
        c1 = t
        for L in self.c2:
            t = L(B, t.shape[1], t.shape[2], t)
        c2 = t
        out = {"stage1": self.out1(B, c2.shape[1], c2.shape[2], c2)}
        if self.arch == "fpn":
            f = self.inner1(B, c1.shape[1], c1.shape[2], c1, res_post=c2, post_up=2)
            out["stage2"] = self.out2(B, f.shape[1], f.shape[2], f)
            if self.num_stage == 3:
                # out3(up2(f) + inner2(c0)) without the 32-channel full-resolution sum (fpn_top_layers)
                lib = self.top_c0._lib
                if self.top_fused is not None and h == 2 * f.shape[1] and w == 2 * f.shape[2]:
                    ap, bc, ws = self.top_fused
                    if ap.device != c0.device:
                        self.top_fused = ap, bc, ws = ap.to(c0.device), bc.to(c0.device), ws
                    o3 = torch.empty(B, h, w, 8, device=c0.device, dtype=c0.dtype)
                    if ws is None:
                        check(lib.damvs_fpn_top_forward(_capi.stream_ptr(c0.device), B, h, w, ptr(c0), ptr(f), ptr(ap),
                                                        ptr(bc), ptr(o3)))
                    else:
                        check(lib.damvs_fpn_top_forward_f32(_capi.stream_ptr(c0.device), B, h, w, ptr(c0), ptr(f),
                                                            ptr(ap), ws, ptr(bc), ptr(o3)))
                else:
                    t = self.top_up(B, f.shape[1], f.shape[2], f)
                    o3 = self.top_c0(B, h, w, c0, res_pre=t)
                check(lib.damvs_conv2d_border_bias(_capi.stream_ptr(o3.device), DTYPES[o3.dtype], B, h, w, o3.shape[3],
                                                   self.top_c0.cout, _capi.float_ptr(self.top_corr), ptr(o3)))
                out["stage3"] = o3
            return out
        f = c2
        for i, (dec, conv) in enumerate(self.up):
            skip = c1 if i == 0 else c0
            y = dec(B, f.shape[1], f.shape[2], f)
            f = conv(B, y.shape[1], y.shape[2], y, skip)
            key = "stage%d" % (i + 2)
            L = self.out2 if i == 0 else self.out3
            out[key] = L(B, f.shape[1], f.shape[2], f)
        return out


class _HipGeoBlock:
    """BasicBlockGeo: conv1(cat(x, g1)) -> ReLU -> conv2(cat(g2, .)) + downsample(cat(x, g1)) -> ReLU."""

    def __init__(self, blk: GeoBlock, dtype, split=None):
        cin = blk.conv1.in_channels - 1
        if split is None:
            x_in = dict(c0=cin)
        else:  # x is torch.cat([a, b]) of two tensors
            x_in = dict(c0=split[0], c0_at=0, c1=split[1], c1_at=split[0])
        self.conv1 = HipConv2d(blk.conv1, dtype, True, geo_at=(cin,), **x_in)
        cout = blk.conv2.out_channels
        self.conv2 = HipConv2d(blk.conv2, dtype, True, c0=cout, c0_at=1, geo_at=(0,))
        self.ds = HipConv2d(blk.downsample[0], dtype, False, geo_at=(cin,), **x_in) if blk.downsample is not None \
            else None
        self.split = split

    def __call__(self, x, g1, g2, post=None):
        xa, xb = x if isinstance(x, tuple) else (x, None)
        B, H, W = xa.shape[:3]
        y = self.conv1(B, H, W, xa, xb, geo=g1)
        idt = self.ds(B, H, W, xa, xb, geo=g1) if self.ds is not None else xa
        return self.conv2(B, y.shape[1], y.shape[2], y, geo=g2, res_pre=idt, res_post=post)


class HipGeoFeatureFusion:
    """GeoFeatureFusion ('z' encoding, 'basic' mask) on libdamvs; stage_idx 1 or 2."""

    def __init__(self, geo, dtype):
        self.mask_type = geo.mask_type
        self.add_origin = geo.add_origin_feat_flag
        D = lambda seq, relu=True: HipConv2d(seq[0], dtype, relu, c0=seq[0].in_channels)
        G = lambda b, split=None: _HipGeoBlock(b, dtype, split)
        self.rgb_init = HipConv2d(geo.rgb_conv_init[0], dtype, True, geo_at=(0, 1, 2, 3))
        self.rgb_enc = [G(getattr(geo, "rgb_encoder_layer%d" % i)) for i in range(1, 6)]
        self.rgb_dec4, self.rgb_dec2 = D(geo.rgb_decoder_layer4), D(geo.rgb_decoder_layer2)
        self.rgb_dec0, self.rgb_dec = D(geo.rgb_decoder_layer0), D(geo.rgb_decoder_layer)
        self.rgb_out = D(geo.rgb_decoder_output)
        self.depth_init = HipConv2d(geo.depth_conv_init[0], dtype, True, geo_at=(0, 1))
        self.dl1, self.dl2 = G(geo.depth_layer1), G(geo.depth_layer2)
        self.dl3 = G(geo.depth_layer3, split=(32, 32))
        self.dl4 = G(geo.depth_layer4)
        self.dl5 = G(geo.depth_layer5, split=(128, 128))
        self.dec = {i: D(getattr(geo, "decoder_layer%d" % i)) for i in range(3, 8)}
        self.rgbdepth = {1: D(geo.rgbdepth_decoder_stage2), 2: D(geo.rgbdepth_decoder_stage3)}
        self.final = {1: D(geo.final_decoder_stage2), 2: D(geo.final_decoder_stage3)}

    def __call__(self, rgb, depth, confidence, depth_values, stage_idx, origin_feat):
        """rgb (B,3,h,w), depth/confidence (B,1,h,w) fp32; origin_feat NHWC (B,h,w,C). Returns NHWC."""
        mask = None
        if self.mask_type != "basic":
            dmin = depth_values[:, 0, None, None, None]
            d = (depth - dmin) / (depth_values[:, -1, None, None, None] - dmin)
            mask = torch.logical_and(d > 0, confidence > confidence.mean()).float()
        pyr = sparse_depth_pyramid(depth, depth_values, mask)
        P = {k: planes(v) for k, v in zip(("d", "d2", "d3", "d4"), pyr)}
        B, _, h, w = rgb.shape
        r0 = self.rgb_init(B, h, w, geo=planes(rgb) + P["d"])
        e = self.rgb_enc
        r1 = e[0](r0, P["d"], P["d2"])
        r2 = e[1](r1, P["d2"], P["d2"])
        r3 = e[2](r2, P["d2"], P["d3"])
        r4 = e[3](r3, P["d3"], P["d3"])
        r5 = e[4](r4, P["d3"], P["d4"])
        run = lambda L, x, **k: L(B, x.shape[1], x.shape[2], x, **k)
        r4p = run(self.rgb_dec4, r5, res_post=r4)
        r2p = run(self.rgb_dec2, r4p, res_post=r2)
        r0p = run(self.rgb_dec0, r2p, res_post=r1)
        rp = run(self.rgb_dec, r0p, res_post=r0)
        rgb_out = run(self.rgb_out, rp)
        rgb_depth = rgb_out[..., 0].float().contiguous()  # (B, h, w) plane
        s0 = self.depth_init(B, h, w, geo=P["d"] + [(rgb_depth, h * w)])
        s1 = self.dl1(s0, P["d"], P["d2"])
        s2 = self.dl2(s1, P["d2"], P["d2"])
        s3 = self.dl3((r2p, s2), P["d2"], P["d3"])
        s4 = self.dl4(s3, P["d3"], P["d3"])
        fusion3 = self.dl5((r4p, s4), P["d3"], P["d4"], post=r5)        # r5 + s5
        fusion4 = run(self.dec[3], fusion3, res_post=s4)                # s4 + dec3
        dec4 = run(self.dec[4], fusion4)
        dec5 = run(self.dec[5], dec4)
        post_origin = origin_feat if self.add_origin else None
        if stage_idx == 1:
            fusion6 = run(self.dec[6], dec5, res_post=s1)               # s1 + dec6
            f = run(self.rgbdepth[1], fusion6, res_post=post_origin)
            return run(self.final[1], f)
        if stage_idx == 2:
            dec6 = run(self.dec[6], dec5)
            fusion7 = run(self.dec[7], dec6, res_post=s0)               # s0 + dec7
            f = run(self.rgbdepth[2], fusion7, res_post=post_origin)
            return run(self.final[2], f)
        raise ValueError("GeoFeatureFusion runs at stage_idx 1 or 2, got %r" % (stage_idx,))
