"""Drop-in ``CascadeMVSNet`` (models/cas_mvsnet.py:137-319) on the MI355X engine.

Same constructor arguments (including the misspelt ``depth_interals_ratio``), the same
``state_dict`` keys (reference checkpoints load with strict=True, test_uni.py:223-224) and the
same ``forward(imgs, proj_matrices, depth_values, intrinsics_matrices)`` -> dict (per-stage dicts
plus the last stage's keys at top level). Two extra keyword arguments select precision:

* ``compute_dtype``  storage of features / cost volumes in the HIP path: torch.float32 (parity
  path, exact-f32 MFMA) or torch.bfloat16 (bf16 MFMA, fp32 accumulate, fp32 regression).
* ``frontend_dtype`` storage dtype of the 2D front-end (FeatureNet, GeoFeatureFusion; default
  float32), and ``frontend_impl``: "hip" (default) runs it on libdamvs's fused NHWC conv2d kernels
  (frontend_hip.py), "torch" on PyTorch-ROCm/MIOpen as BN-folded channels-last copies (A/B only).
  The reference-keyed modules keep the parameters/state_dict either way.

Per stage: hypotheses (HIP) -> [GeoFeatureFusion, stages 2/3] -> DepthNet (HIP). The reference's
host syncs (depth_values .cpu(), :191-193; stage-3 debug prints, :275-285) are not reproduced.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .depthnet import DepthNet
from .engine import hypotheses
from .frontend import FeatureNet, GeoFeatureFusion, ConvBNReLU2d
from .frontend_fold import fold_frontend
from .layers import CostRegNet

STAGE_SCALE = {"stage1": 4, "stage2": 2, "stage3": 1}


class RefineNet(nn.Module):
    """Key holder for models/module.py:594-606 (its forward is broken in the reference: F.cat)."""

    def __init__(self):
        super().__init__()
        self.conv1 = ConvBNReLU2d(4, 32, 3, 1, 1)
        self.conv2 = ConvBNReLU2d(32, 32, 3, 1, 1)
        self.conv3 = ConvBNReLU2d(32, 32, 3, 1, 1)
        self.res = ConvBNReLU2d(32, 1, 3, 1, 1)


_SIDE_STREAMS = {}  # device index -> sub-batch streams shared by all models (CascadeMVSNet._side_streams)

class CascadeMVSNet(nn.Module):
    def __init__(self, refine=False, ndepths=[64, 32, 8], depth_interals_ratio=[4, 2, 1], share_cr=False,
                 grad_method="detach", arch_mode="fpn", cr_base_chs=[8, 8, 8], agg_mode="adaptive",
                 compute_dtype=torch.float32, frontend_dtype=None, frontend_impl="hip"):
        super().__init__()
        assert len(ndepths) == len(depth_interals_ratio)
        if len(ndepths) != 3:
            raise NotImplementedError("the reference wires GeoFeatureFusion for exactly 3 stages")
        self.refine, self.share_cr = refine, share_cr
        self.ndepths, self.depth_interals_ratio = list(ndepths), list(depth_interals_ratio)
        self.grad_method, self.arch_mode, self.cr_base_chs = grad_method, arch_mode, list(cr_base_chs)
        self.num_stage = len(ndepths)
        self.stage_infos = {k: {"scale": float(v)} for k, v in STAGE_SCALE.items()}
        self.compute_dtype = compute_dtype
        self.frontend_dtype = frontend_dtype
        if frontend_impl not in ("hip", "torch"):
            raise ValueError("frontend_impl must be 'hip' or 'torch'")
        self.frontend_impl = frontend_impl

        self.feature = FeatureNet(base_channels=8, stride=4, num_stage=self.num_stage, arch_mode=arch_mode)
        self.GeoFeatureFusionNet = GeoFeatureFusion(convolutional_layer_encoding="z", mask_type="basic",
                                                    add_origin_feat_flag=True)
        self.geo_reg_encodings = ["std", "z", "z", "z"]
        if share_cr:
            self.cost_regularization = CostRegNet(in_channels=self.feature.out_channels, base_channels=8)
        else:
            self.cost_regularization = nn.ModuleList(
                [CostRegNet(in_channels=self.feature.out_channels[i], base_channels=self.cr_base_chs[i])
                 for i in range(self.num_stage)])
        if refine:
            self.refine_network = RefineNet()
        self.DepthNet = DepthNet(agg_mode, self.feature.out_channels, compute_dtype=compute_dtype)
        self._folded_key = None

    def _frontend(self):
        """Front-end executors, rebuilt whenever FeatureNet / GeoFeatureFusion parameters change
        (load_state_dict bumps tensor versions): BN-folded copies, then either fused HIP conv2d layer
        chains ("hip") or channels-last ``frontend_dtype`` module copies ("torch")."""
        fd = self.frontend_dtype or torch.float32
        mods = (self.feature, self.GeoFeatureFusionNet)
        ver = tuple(t._version for m in mods for t in list(m.parameters()) + list(m.buffers()))
        key = (ver, fd, self.frontend_impl, str(next(self.feature.parameters()).device))
        if getattr(self, "_folded_key", None) != key:
            if self.frontend_impl == "hip":
                from .frontend_hip import HipFeatureNet, HipGeoFeatureFusion
                f32 = tuple(fold_frontend(m, torch.float32) for m in mods)
                self._folded = (HipFeatureNet(f32[0], fd), HipGeoFeatureFusion(f32[1], fd))
            else:
                self._folded = tuple(fold_frontend(m, fd) for m in mods)
            self._folded_key = key
        return self._folded

    def _apply(self, fn, *a, **k):
        self._folded_key = None
        return super()._apply(fn, *a, **k)

    def extract_features(self, imgs):
        """FeatureNet over all views in one batched call (BN in eval is per-sample). Returns per view a
        dict of stage features: NHWC (B,h,w,C) for the HIP front-end, NCHW views for "torch"."""
        feat, _ = self._frontend()
        B, N = imgs.shape[:2]
        if self.frontend_impl == "hip":
            f = feat(imgs)  # view-major rows: view v = rows v*B.. (the images are read in place)
            return [{k: v[i * B:(i + 1) * B] for k, v in f.items()} for i in range(N)]
        x = imgs.reshape(B * N, *imgs.shape[2:]).contiguous(memory_format=torch.channels_last)
        f = feat(x)
        return [{k: v.reshape(B, N, *v.shape[1:])[:, i] for k, v in f.items()} for i in range(N)]

    def _side_streams(self, n, device):
        """The sub-batch streams, one process-wide set per device shared by every model: torch.cuda.Stream() hands out
        the next stream of PyTorch's pool, and HIP places streams on its hardware queues in creation order, so a second
        model with streams of its own could land a sub-batch on the main stream's queue (measured: whichever of the
        bf16 and fp32 models ran second in one bench process lost 10-14 %, the fp32 parity path 78 against 86 maps/s)."""
        key = torch.device(device).index if torch.device(device).index is not None else torch.cuda.current_device()
        pool = _SIDE_STREAMS.get(key)
        if pool is None or len(pool) < n:
            pool = (pool or []) + [torch.cuda.Stream(device) for _ in range(n - len(pool or []))]
            _SIDE_STREAMS[key] = pool
        return pool[:n]

    def _forward_streams(self, imgs, proj_matrices, depth_values, intrinsics_matrices, nstreams, check_range=True,
                         offset=None):
        """The batch as ``nstreams`` sub-batches of reference views on concurrent HIP streams, merged along the
        batch. Per sample every kernel sees the same inputs as in one batch, so the outputs are bitwise those of
        the single-stream forward (tests/test_gpu_streams.py); the gain is overlap between kernels with different
        bounds (one sub-batch's TA-bound warp beside another's HBM / MFMA-bound U-Net or front-end).
        ``offset``: a stage-hook name ("stage1.hypotheses", ...); sub-batch i + 1 then starts when sub-batch i reaches
        that point of its forward (an event on its stream), so the sub-batches run different layers side by side."""
        B = imgs.shape[0]
        cut = [B * i // nstreams for i in range(nstreams + 1)]
        main = torch.cuda.current_stream(imgs.device)

        def part(x, a, b):
            if isinstance(x, dict):
                return {k: part(v, a, b) for k, v in x.items()}
            return x[a:b] if isinstance(x, torch.Tensor) else x

        pool = self._side_streams(nstreams, imgs.device)
        outs = []
        gate = None  # the previous sub-batch's event at `offset`
        for st, a, b in zip(pool, cut[:-1], cut[1:]):
            st.wait_stream(main)
            if gate is not None:
                st.wait_event(gate)
            mark = {}

            def hook(name, st=st, mark=mark):
                if name == offset:
                    mark["ev"] = torch.cuda.Event()
                    mark["ev"].record(st)

            with torch.cuda.stream(st):
                outs.append(self.forward(part(imgs, a, b), part(proj_matrices, a, b), part(depth_values, a, b),
                                         part(intrinsics_matrices, a, b), check_range=False,
                                         stage_hook=hook if offset else None))
            gate = mark.get("ev")

        # batch-sized outputs allocated on the main stream, each stream copying its rows right after its own
        # forward (the copies overlap the other sub-batches' kernels instead of following all of them)
        memo = {}  # the top-level keys alias the last stage's tensors: one batch tensor (and copy) each

        def alloc(v):
            if isinstance(v, dict):
                return {k: alloc(x) for k, x in v.items()}
            if isinstance(v, torch.Tensor):
                if id(v) not in memo:
                    memo[id(v)] = torch.empty((B,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
                return memo[id(v)]
            return v

        full = alloc(outs[0])

        def fill(dst, src, a, b, st, done):
            if isinstance(dst, dict):
                for k in dst:
                    fill(dst[k], src[k], a, b, st, done)
            elif isinstance(dst, torch.Tensor) and id(dst) not in done:
                done.add(id(dst))
                dst[a:b].copy_(src)
                dst.record_stream(st)

        for i, (st, a, b) in enumerate(zip(pool, cut[:-1], cut[1:])):
            st.wait_stream(main)  # after the allocations (their blocks may come from pending main-stream work)
            with torch.cuda.stream(st):
                fill(full, outs[i], a, b, st, set())
        for st in pool:
            main.wait_stream(st)
        if check_range:  # after every sub-batch is enqueued: one host sync for the whole forward
            self.DepthNet.check_range()
        return full

    def forward(self, imgs, proj_matrices, depth_values, intrinsics_matrices=None, stage_hook=None, depthnet=None,
                streams=1, check_range=True, stream_offset="auto"):
        """``depthnet``: optional stage runner (stage_idx, NHWC features, proj, hyps, cost_regularization) -> dict,
        e.g. sharded.DepthShardedDepthNet (one depth map over several GPUs); default: this model's DepthNet.
        ``streams`` > 1 runs the batch as that many sub-batches on concurrent streams (_forward_streams; not with
        a stage hook or a custom stage runner; ``stream_offset``: see _forward_streams; "auto": "stage1.hypotheses" for
        fp32 storage, none for bf16 -- the measured best, profiles/r06/ab_rs2_offset_r06t: fp32 102.4-102.7 ->
        103.1-103.3 maps/s, bf16 205.6 -> 203.7). ``check_range``: after the last stage, read every stage's range
        status (damvs_stage_status, one host sync per forward) and raise damvsnet_amd._capi.DamvsRangeError if any
        depth / confidence / variance is non-finite. With a custom ``depthnet`` runner the range status is that
        runner's business: sharded.DepthShardedDepthNet runs the stage as split layer calls, which do not write a
        status word, so no DamvsRangeError is raised on that path."""
        if streams > 1 and imgs.shape[0] > 1 and stage_hook is None and depthnet is None and imgs.is_cuda \
                and not self.refine:
            if stream_offset == "auto":
                stream_offset = "stage1.hypotheses" if self.compute_dtype == torch.float32 else None
            return self._forward_streams(imgs, proj_matrices, depth_values, intrinsics_matrices,
                                         min(int(streams), imgs.shape[0]), check_range, stream_offset)
        if self.refine:
            raise NotImplementedError("refine=True: the reference RefineNet forward is not runnable "
                                      "(models/module.py:602 calls F.cat)")
        if not imgs.is_cuda:
            raise ValueError("damvsnet_amd is a GPU engine: move the model and inputs to a HIP device")
        hook = stage_hook or (lambda name: None)
        B, N, _, H, W = imgs.shape
        hook("features")
        features = self.extract_features(imgs)
        outputs = {}
        depth = exp_var = conf = None
        for s in range(self.num_stage):
            name = "stage%d" % (s + 1)
            scale = STAGE_SCALE[name]
            fs = [f[name] for f in features]
            if s >= 1:
                hook(name + ".geofusion")
                _, geo = self._frontend()
                # scale 1 (stage 3) is the identity (source index (x + 0.5) - 0.5 = x): read imgs[:, 0] in place
                ref_img = imgs[:, 0] if s == 2 and self.frontend_impl == "hip" else \
                    F.interpolate(imgs[:, 0], scale_factor=1.0 / 2 ** (2 - s), mode="bilinear", align_corners=False)
                dl = F.interpolate(depth.unsqueeze(1), scale_factor=2, mode="bilinear", align_corners=False)
                cl = F.interpolate(conf.unsqueeze(1), scale_factor=2, mode="bilinear", align_corners=False)
                if self.frontend_impl == "hip":
                    fs[0] = geo(ref_img, dl, cl, depth_values, s, fs[0])
                else:
                    fs[0] = geo(ref_img.contiguous(memory_format=torch.channels_last), dl, cl, depth_values, s,
                                fs[0], None if intrinsics_matrices is None else intrinsics_matrices[name])
            hook(name + ".hypotheses")
            hyps = hypotheses(depth_values, self.ndepths[s], H, W, scale, depth, exp_var)
            hook(name + ".depthnet")
            cr = self.cost_regularization if self.share_cr else self.cost_regularization[s]
            if depthnet is not None:
                if self.frontend_impl != "hip":
                    raise ValueError("a custom stage runner takes the HIP front-end's NHWC features")
                out = depthnet(s, fs, proj_matrices[name], hyps, cr)
            elif self.frontend_impl == "hip":
                out = self.DepthNet.forward_nhwc(s, fs, proj_matrices[name], hyps, cr)
            else:
                out = self.DepthNet(s, fs, proj_matrices[name], hyps, self.ndepths[s], cr, check_range=False)
            depth, conf, exp_var = out["depth"], out["photometric_confidence"], out["variance"]
            outputs[name] = out
            outputs.update(out)
        hook("end")
        if check_range and depthnet is None:
            self.DepthNet.check_range()
        return outputs
