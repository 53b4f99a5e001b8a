"""Drop-in ``DepthNet`` and ``homo_warping`` backed by libdamvs.so.

Mirrors the reference interfaces (same names, argument meaning, output dict, error behaviour):

* ``DepthNet(mode, in_channels).forward(stage_idx, features, proj_matrices, depth_values, num_depth,
  cost_regularization, prob_volume_init=None)``  — models/cas_mvsnet.py:10-134
* ``homo_warping(src_fea, src_proj, ref_proj, depth_values)``  — models/module.py:297-332

Inputs are the reference's NCHW/NCDHW tensors on a HIP device. Features are handed to the
kernels as NHWC: a channels-last NCHW tensor already has that memory, so no copy is made for
the front-end's outputs. Inference only (the reference's DepthNet is used under
``torch.no_grad()`` by test_uni.py:229); there is no eager/CPU fallback.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _capi
from .engine import StageEngine, DTYPES, hypotheses, proj_prepare  # noqa: F401
from .layers import AggWeightNetVolume
from ._capi import check, ptr


def to_nhwc(t: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """(B,C,h,w) -> contiguous (B,h,w,C) of ``dtype``; free for channels-last inputs."""
    x = t.permute(0, 2, 3, 1)
    if x.dtype != dtype:
        x = x.to(dtype)
    return x.contiguous()


def _require_gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("damvsnet_amd is a GPU engine: inputs must be on a HIP device (got %s)" % t.device)


class DepthNet(nn.Module):
    def __init__(self, mode="adaptive", in_channels=None, compute_dtype=torch.float32):
        super().__init__()
        self.mode = mode
        assert mode in ("variance", "adaptive"), "Don't support {}!".format(mode)
        if self.mode == "adaptive":
            self.weight_net = nn.ModuleList([AggWeightNetVolume(c) for c in in_channels])
        self.compute_dtype = compute_dtype
        self._engines = {}
        self.probe = None  # optional callable(stage_idx) -> 4 torch.cuda.Event (bench.py in-pipeline timing)

    def engine(self, stage_idx, cost_regularization, device):
        aggw = self.weight_net[stage_idx] if self.mode == "adaptive" else None
        key = (stage_idx, id(cost_regularization), str(device), self.compute_dtype)
        eng = self._engines.get(key)
        ver = tuple(t._version for t in list(cost_regularization.parameters()) + list(cost_regularization.buffers()))
        if aggw is not None:
            ver += tuple(t._version for t in list(aggw.parameters()) + list(aggw.buffers()))
        if eng is None or eng.version != ver:
            eng = StageEngine(cost_regularization, aggw, self.mode, self.compute_dtype, device)
            self._engines[key] = eng
        return eng

    def _apply(self, fn, *a, **k):  # .to()/.cuda() invalidate packed weights
        self._engines = {}
        return super()._apply(fn, *a, **k)

    def check_range(self):
        """Raise damvsnet_amd._capi.DamvsRangeError when a stage forward since the last check produced non-finite
        depth / confidence / variance (the fp32 path's split-f16 products are limited to |x| < 65520; the reference's
        fp32 convolutions are not). Synchronises the streams those forwards ran on."""
        err = None
        for eng in list(self._engines.values()):  # every engine's status is read (and cleared) before raising
            try:
                eng.check_range()
            except Exception as e:  # noqa: BLE001 (re-raised below)
                err = err or e
        if err is not None:
            raise err

    def forward(self, stage_idx, features, proj_matrices, depth_values, num_depth, cost_regularization,
                prob_volume_init=None, return_prob_volume=True, check_range=True):
        """The reference's per-stage call (models/cas_mvsnet.py:18). ``check_range`` (default on, one host sync):
        raise DamvsRangeError right away on non-finite outputs; CascadeMVSNet passes False and checks once per
        forward."""
        assert len(features) == proj_matrices.shape[1], "Different number of images and projection matrices"
        assert depth_values.shape[1] == num_depth, "depth_values.shape[1]:{}  num_depth:{}".format(
            depth_values.shape[1], num_depth)
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()) and self.training:
            raise NotImplementedError("damvsnet_amd is an inference engine; wrap the call in torch.no_grad()")
        _require_gpu(depth_values, proj_matrices, *features)
        feats = [to_nhwc(f, self.compute_dtype) for f in features]
        return self.forward_nhwc(stage_idx, feats, proj_matrices, depth_values, cost_regularization,
                                 prob_volume_init, return_prob_volume, check_range=check_range)

    def forward_nhwc(self, stage_idx, feats_nhwc, proj_matrices, depth_values, cost_regularization,
                     prob_volume_init=None, return_prob_volume=True, check_range=False):
        """Same as forward() with features already NHWC (B,h,w,C) — the HIP front-end's output. ``check_range``:
        raise DamvsRangeError on non-finite outputs right away (a host sync); CascadeMVSNet checks once per forward."""
        dev = depth_values.device
        eng = self.engine(stage_idx, cost_regularization, dev)
        feats = [f if f.dtype == self.compute_dtype and f.is_contiguous() else f.to(self.compute_dtype).contiguous()
                 for f in feats_nhwc]
        hyps = depth_values.float().contiguous()
        pinit = prob_volume_init.float().contiguous() if prob_volume_init is not None else None
        depth, conf, var, prob = eng.forward(feats, proj_matrices.float().contiguous(), hyps, pinit,
                                             want_prob=return_prob_volume,
                                             probe=self.probe(stage_idx) if self.probe is not None else None)
        if check_range:
            eng.check_range()
        return {"depth": depth, "photometric_confidence": conf, "variance": var, "prob_volume": prob,
                "depth_values": depth_values}


def homo_warping(src_fea, src_proj, ref_proj, depth_values, compute_dtype=None):
    """Warp ``src_fea`` (B,C,H,W) into the reference frustum at ``depth_values`` ((B,D) or (B,D,H,W)).

    ``src_proj``/``ref_proj`` are composed 4x4 projections (models/cas_mvsnet.py:44-47). Returns
    (B,C,D,H,W) (memory NDHWC). Any C: channels are zero-padded to a multiple of 8 and warped in
    kernel-sized slices of 32/16/8 channels.
    """
    lib = _capi.load_library()
    _require_gpu(src_fea, src_proj, ref_proj, depth_values)
    B, C, H, W = src_fea.shape
    D = depth_values.shape[1]
    dt = compute_dtype or (torch.bfloat16 if src_fea.dtype == torch.bfloat16 else torch.float32)
    if depth_values.dim() == 2:
        depth_values = depth_values.view(B, D, 1, 1).expand(B, D, H, W)
    hyps = depth_values.float().contiguous()
    eye = torch.eye(3, device=src_fea.device, dtype=torch.float32)
    pair = torch.zeros(B, 2, 2, 4, 4, device=src_fea.device, dtype=torch.float32)
    pair[:, 0, 0] = ref_proj.float()
    pair[:, 1, 0] = src_proj.float()
    pair[:, :, 1, :3, :3] = eye  # K = I: the pair is already composed
    rt = proj_prepare(pair)
    Cp = (C + 7) // 8 * 8
    src = to_nhwc(src_fea, dt)
    if Cp != C:
        src = torch.nn.functional.pad(src, (0, Cp - C))
    slices, c0 = [], 0
    while c0 < Cp:
        cc = next(s for s in (32, 16, 8) if s <= Cp - c0)
        slices.append((c0, cc))
        c0 += cc
    outs = []
    for c0, cc in slices:
        part = src if len(slices) == 1 else src[..., c0:c0 + cc].contiguous()
        o = torch.empty(B, D, H, W, cc, device=src_fea.device, dtype=dt)
        check(lib.damvs_homo_warp(_capi.stream_ptr(src_fea.device), DTYPES[dt], B, cc, D, H, W, ptr(part), ptr(rt),
                                  ptr(hyps), ptr(o)))
        outs.append(o)
    out = outs[0] if len(outs) == 1 else torch.cat(outs, dim=-1)
    return out[..., :C].permute(0, 4, 1, 2, 3)
