"""Host-side engine: owns one ``damvs_stage`` per (cascade stage, device, dtype) and launches the
per-stage hot path through the C ABI on PyTorch's current HIP stream.

PyTorch is plumbing here: device buffers come from its caching allocator and the stream is
its current stream; all compute of the hot path happens in libdamvs.so.
"""
from __future__ import annotations

import ctypes

import torch

from . import _capi
from ._capi import check, ptr

DTYPES = {torch.float32: _capi.DAMVS_F32, torch.bfloat16: _capi.DAMVS_BF16}


def _host(t):
    return t.detach().to("cpu", torch.float32).contiguous()


def _param_version(mod):
    return tuple(t._version for t in list(mod.parameters()) + list(mod.buffers()))


class StageEngine:
    """Folded, packed weights of one stage (CostRegNet + weight net) resident on one device."""

    def __init__(self, costreg, aggw, agg_mode: str, dtype: torch.dtype, device: torch.device):
        lib = _capi.load_library()
        if dtype not in DTYPES:
            raise TypeError("compute dtype must be float32 or bfloat16, got %r" % (dtype,))
        self.dtype, self.device, self.C, self.base = dtype, device, costreg.in_channels, costreg.base_channels
        self.mode = _capi.DAMVS_AGG_ADAPTIVE if agg_mode == "adaptive" else _capi.DAMVS_AGG_VARIANCE
        keep = []  # host tensors must outlive the create call

        def h(t):
            t = _host(t)
            keep.append(t)
            return t.data_ptr()

        def bn(m):
            return _capi.DamvsBN(h(m.weight), h(m.bias), h(m.running_mean), h(m.running_var), float(m.eps))

        layers = [getattr(costreg, n) for n in costreg.ENCODER + costreg.DECODER]
        cp = _capi.DamvsCostregParams()
        cp.in_channels, cp.base_channels = costreg.in_channels, costreg.base_channels
        for i, m in enumerate(layers):
            cp.conv_weight[i] = h(m.conv.weight)
            cp.bn[i] = bn(m.bn)
        cp.prob_weight = h(costreg.prob.weight)
        ap = None
        if self.mode == _capi.DAMVS_AGG_ADAPTIVE:
            w0, w1 = aggw.w_net[0], aggw.w_net[1]
            ap = _capi.DamvsAggweightParams(aggw.in_channels, h(w0.conv.weight), bn(w0.bn), h(w1.conv.weight), bn(w1.bn))
        handle = ctypes.c_void_p()
        with torch.cuda.device(device):
            check(lib.damvs_stage_create(ctypes.byref(cp), ctypes.byref(ap) if ap is not None else None, self.mode,
                                         DTYPES[dtype], ctypes.byref(handle)))
        self.handle = handle
        self._lib = lib
        self._ws = None
        self._unchecked = {}  # stream pointer -> {data_ptr: workspace} of forwards whose range status was not read yet
        self.version = _param_version(costreg) + (_param_version(aggw) if aggw is not None else ())

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                self._lib.damvs_stage_destroy(h)
            except Exception:
                pass

    def workspace(self, B, N, D, h, w):
        """The stage's scratch, one buffer per stream (sub-batches running on concurrent streams each
        get their own; a buffer is reused by later calls on its stream, which are ordered after it)."""
        n = ctypes.c_size_t()
        check(self._lib.damvs_stage_workspace_size(self.handle, B, N, D, h, w, ctypes.byref(n)))
        if self._ws is None:
            self._ws = {}
        key = _capi.stream_ptr(self.device)
        ws = self._ws.get(key)
        if ws is None or ws.numel() < n.value:
            ws = self._ws[key] = torch.empty(n.value, dtype=torch.uint8, device=self.device)
            ws[:4].zero_()  # the range status word (damvs_stage_status)
        return ws

    def forward(self, feats_nhwc, proj, hyps, prob_init=None, want_prob=True, probe=None):
        """feats_nhwc: list of N (B,h,w,C) tensors of self.dtype; proj (B,N,2,4,4); hyps (B,D,h,w) float32.
        probe: None or 4 torch.cuda.Event recorded before / after the warp, after the U-Net, after the regression."""
        N = len(feats_nhwc)
        B, h, w, C = feats_nhwc[0].shape
        D = hyps.shape[1]
        dev = self.device
        ws = self.workspace(B, N, D, h, w)
        depth = torch.empty(B, h, w, device=dev, dtype=torch.float32)
        conf = torch.empty_like(depth)
        var = torch.empty_like(depth)
        prob = torch.empty(B, D, h, w, device=dev, dtype=torch.float32) if want_prob else None
        fptrs = (ctypes.c_void_p * N)(*[f.data_ptr() for f in feats_nhwc])
        # a workspace replaced by a larger one (shape change between checks) stays pending until check_range()
        self._unchecked.setdefault(_capi.stream_ptr(dev), {})[ws.data_ptr()] = ws
        if probe is None:
            check(self._lib.damvs_stage_forward(self.handle, _capi.stream_ptr(dev), B, N, D, h, w, fptrs, ptr(proj),
                                                ptr(hyps), ptr(prob_init), ptr(ws), ws.numel(), ptr(depth), ptr(conf),
                                                ptr(var), ptr(prob)))
        else:
            for e in probe:  # torch creates the HIP event at its first record
                e.record()
            evs = (ctypes.c_void_p * 4)(*[e.cuda_event for e in probe])
            check(self._lib.damvs_stage_forward_probed(self.handle, _capi.stream_ptr(dev), B, N, D, h, w, fptrs,
                                                       ptr(proj), ptr(hyps), ptr(prob_init), ptr(ws), ws.numel(),
                                                       ptr(depth), ptr(conf), ptr(var), ptr(prob), evs))
        return depth, conf, var, prob

    def check_range(self):
        """Raise DamvsRangeError if any forward since the last check wrote non-finite depth / confidence / variance
        (damvs_stage_status: sticky per workspace until read; synchronises the streams those forwards ran on)."""
        pending, self._unchecked = self._unchecked, {}
        err = None
        for stream, wss in pending.items():  # every status is read (and cleared) before the first error is raised
            for ws in wss.values():
                try:
                    check(self._lib.damvs_stage_status(self.handle, stream, ptr(ws), ws.numel()))
                except _capi.DamvsError as e:
                    err = err or e
        if err is not None:
            raise err

    # ---- split entry points (parity tests / sharded execution)
    def warp_aggregate(self, feats, proj, hyps, rt=None, layout=_capi.DAMVS_LAYOUT_NHWC, out=None):
        """feats: N NHWC (B,h,w,C) tensors, or channel-blocked ones (see block_channels) with
        layout=DAMVS_LAYOUT_CBLOCK; rt from proj_prepare (computed from proj when None); out: the (B,D,h,w,C)
        volume to write (allocated when None)."""
        N = len(feats)
        B, D, h, w = hyps.shape
        C = self.C
        if rt is None:
            rt = proj_prepare(proj)
        vol = torch.empty(B, D, h, w, C, device=self.device, dtype=self.dtype) if out is None else out
        if vol.shape != (B, D, h, w, C) or vol.dtype != self.dtype or not vol.is_contiguous():
            raise ValueError("warp_aggregate: out must be a contiguous %s tensor of shape %s" % (self.dtype, (B, D, h, w, C)))
        fptrs = (ctypes.c_void_p * N)(*[f.data_ptr() for f in feats])
        check(self._lib.damvs_warp_aggregate(self.handle, _capi.stream_ptr(self.device), B, N, D, h, w, fptrs, layout,
                                             ptr(rt), ptr(hyps), ptr(vol)))
        return vol

    def warp_aggregate_rows(self, feats, rt, hyps, h, y0, rows, out_y, out, layout=_capi.DAMVS_LAYOUT_NHWC):
        """Aggregated volume of reference rows [y0, y0 + rows) from the whole feature maps (h rows), read from
        hyps [B][D][R][w] and written to out [B][D][R][w][C] at rows [out_y, out_y + rows) (R = hyps.shape[2]);
        bitwise the same voxels as warp_aggregate."""
        N = len(feats)
        B, D, R, w = hyps.shape
        fptrs = (ctypes.c_void_p * N)(*[f.data_ptr() for f in feats])
        check(self._lib.damvs_warp_aggregate_rows(self.handle, _capi.stream_ptr(self.device), B, N, D, h, w, y0, rows,
                                                  R, out_y, fptrs, layout, ptr(rt), ptr(hyps), ptr(out)))
        return out

    def unet_layer(self, layer, D, h, w, inp, out, in_slot=None, out_slot=None):
        """CostRegNet layer ``layer`` (0..9 = conv0..conv6, conv7, conv9, conv11) of a level-0 volume of
        D x h x w; deconvs add into ``out`` in place (it holds the skip tensor). ``in_slot`` / ``out_slot``: fp32
        magnitude slots (new_slots rows) of the input / output tensor (damvs_costreg_layer_scaled); None: unscaled /
        not recorded."""
        B = inp.shape[0]
        check(self._lib.damvs_costreg_layer_scaled(self.handle, _capi.stream_ptr(self.device), layer, B, D, h, w,
                                                   ptr(inp), ptr(out), ptr(in_slot), ptr(out_slot)))
        return out

    # ---- fp32 magnitude slots for layer-by-layer execution (include/damvs.h DAMVS_AMAX_SLOT_BYTES)
    SLOT_WORDS = 1024  # DAMVS_AMAX_SLOT_BYTES / 4

    def new_slots(self, B, n=10):
        """Zeroed magnitude slots of n tensors x B batch elements: int32 [n][B][SLOT_WORDS] on the engine's device
        (slots[i] is tensor i's, one slot per batch element, as damvs_costreg_layer_scaled takes them)."""
        return torch.zeros(n, B, self.SLOT_WORDS, dtype=torch.int32, device=self.device)

    def tensor_amax(self, t, slots):
        """Fold max |t[b]| of a contiguous float32 device tensor [B][...] into slots[b] (damvs_tensor_amax per b)."""
        for b in range(t.shape[0]):
            check(self._lib.damvs_tensor_amax(_capi.stream_ptr(self.device), ptr(t[b]), t[b].numel(), ptr(slots[b])))
        return slots

    def unet_buffers(self, B, D, h, w):
        """Level tensors c0..c6 (conv0..conv6 outputs, NDHWC) of a D x h x w volume."""
        b = self.base
        spec = ((0, b), (1, 2 * b), (1, 2 * b), (2, 4 * b), (2, 4 * b), (3, 8 * b), (3, 8 * b))
        return [torch.empty(B, D >> l, h >> l, w >> l, c, device=self.device, dtype=self.dtype) for l, c in spec]

    def regress_c0(self, c0, hyps, prob_init=None, want_prob=True, scratch=None):
        """Prob conv + softmax regression on the U-Net output c0 [B][D][h][w][base] (damvs_stage_regress)."""
        B, D, h, w, _ = c0.shape
        dev = self.device
        depth = torch.empty(B, h, w, device=dev, dtype=torch.float32)
        conf, var = torch.empty_like(depth), torch.empty_like(depth)
        prob = torch.empty(B, D, h, w, device=dev, dtype=torch.float32) if want_prob else None
        if scratch is None:
            scratch = torch.empty(B, D, h, w, device=dev, dtype=torch.float32)
        check(self._lib.damvs_stage_regress(self.handle, _capi.stream_ptr(dev), B, D, h, w, ptr(c0), ptr(hyps),
                                            ptr(prob_init), ptr(scratch), ptr(depth), ptr(conf), ptr(var), ptr(prob)))
        return depth, conf, var, prob

    def costreg_logits(self, vol):
        B, D, h, w, C = vol.shape
        ws = self.workspace(B, 2, D, h, w)
        logits = torch.empty(B, D, h, w, device=self.device, dtype=torch.float32)
        check(self._lib.damvs_costreg_logits(self.handle, _capi.stream_ptr(self.device), B, D, h, w, ptr(vol), ptr(ws),
                                              ws.numel(), ptr(logits)))
        return logits


def _check_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("damvsnet_amd runs on the GPU only; got a %s tensor" % t.device)


def proj_prepare(proj):
    """(B,N,2,4,4) -> (B,N-1,12) [R|t] of P_src inv(P_ref)."""
    lib = _capi.load_library()
    _check_cuda(proj)
    proj = proj.float().contiguous()
    B, N = proj.shape[:2]
    rt = torch.empty(B, N - 1, 12, device=proj.device, dtype=torch.float32)
    check(lib.damvs_proj_prepare(_capi.stream_ptr(proj.device), B, N, ptr(proj), ptr(rt)))
    return rt


def warp_blocked(C, element_size, N=5):
    """Whether damvs_stage_forward gathers channel-blocked copies of C-channel feature maps at N views: the library's
    own decision (damvs_warp_feat_blocked_n), so split-entry callers lay the maps out exactly as the stage forward
    does."""
    lib = _capi.load_library()
    r = lib.damvs_warp_feat_blocked_n(_capi.DAMVS_BF16 if element_size == 2 else _capi.DAMVS_F32, int(C), int(N))
    check(r if r < 0 else 0)
    return r == 1


def block_channels(feats_nhwc):
    """N NHWC (B,h,w,C) maps -> channel-blocked copies [B][C/E][h][w][E] (E = 16 bytes)."""
    lib = _capi.load_library()
    N = len(feats_nhwc)
    B, h, w, C = feats_nhwc[0].shape
    dt = feats_nhwc[0].dtype
    E = 16 // feats_nhwc[0].element_size()
    outs = [torch.empty(B, C // E, h, w, E, device=f.device, dtype=dt) for f in feats_nhwc]
    src = (ctypes.c_void_p * N)(*[f.data_ptr() for f in feats_nhwc])
    dst = (ctypes.c_void_p * N)(*[o.data_ptr() for o in outs])
    check(lib.damvs_block_channels(_capi.stream_ptr(feats_nhwc[0].device), DTYPES[dt], N, B, h, w, C, src, dst))
    return outs


def regress(logits, hyps, want_prob=True):
    lib = _capi.load_library()
    _check_cuda(logits, hyps)
    B, D, h, w = logits.shape
    logits, hyps = logits.float().contiguous(), hyps.float().contiguous()
    depth = torch.empty(B, h, w, device=logits.device)
    conf, var = torch.empty_like(depth), torch.empty_like(depth)
    prob = torch.empty_like(logits) if want_prob else None
    check(lib.damvs_regress(_capi.stream_ptr(logits.device), B, D, h, w, ptr(logits), ptr(hyps), None, ptr(depth),
                            ptr(conf), ptr(var), ptr(prob)))
    return depth, conf, var, prob


def hypotheses(depth_values, ndepth, H, W, scale, prev_depth=None, prev_var=None):
    """Stage hypotheses (B, ndepth, H/scale, W/scale) — see damvs_hypotheses in include/damvs.h."""
    lib = _capi.load_library()
    dev = depth_values.device
    _check_cuda(depth_values, prev_depth, prev_var)
    B = depth_values.shape[0]
    out = torch.empty(B, ndepth, H // scale, W // scale, device=dev, dtype=torch.float32)
    dv = depth_values.float().contiguous()
    if prev_depth is None:
        check(lib.damvs_hypotheses(_capi.stream_ptr(dev), B, ndepth, H, W, scale, ptr(dv), dv.shape[1], None, None, 0, 0,
                                   ptr(out)))
    else:
        pd, pv = prev_depth.float().contiguous(), prev_var.float().contiguous()
        check(lib.damvs_hypotheses(_capi.stream_ptr(dev), B, ndepth, H, W, scale, ptr(dv), dv.shape[1], ptr(pd), ptr(pv),
                                   pd.shape[-2], pd.shape[-1], ptr(out)))
    return out
