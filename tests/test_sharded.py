"""CPU: depth-sharded execution of one stage (damvsnet_amd/sharded.py) -- the shard, halo, all-to-all and
all-gather bookkeeping -- with a float64 CPU stand-in for the HIP stage engine, against the unsharded oracle
stage (oracle/mvs_oracle.py depthnet_stage, models/cas_mvsnet.py:18-134): in-process (ThreadGroup, P = 1..5,
every warp partitioning, incl. north_star's literal volume all-gather) and over torch.distributed gloo (world 2 and 3, uneven slabs and depth shards).

The stand-in runs each U-Net layer with torch's CPU conv on the whole haloed slab tensor, exactly as the HIP
engine runs its whole-tensor kernel on it, so the sharded result must equal the whole-image one up to float64
summation-order noise (CPU GEMM blocking changes with the tensor height).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

from common import model_state, depthnet_inputs
from oracle import mvs_oracle as O
from damvsnet_amd import sharded as S

LAYERS = ("conv0", "conv1", "conv2", "conv3", "conv4", "conv5", "conv6", "conv7", "conv9", "conv11")
F64 = torch.float64


class CpuStageEngine:
    """Test stand-in for damvsnet_amd.engine.StageEngine: float64 NDHWC tensors on the CPU, the oracle's
    operators. Feature maps and cameras are bound at construction (the sharded code passes them through)."""

    def __init__(self, sd, stage_idx, mode, feats, proj):
        self.sd = {k: (v.to(F64) if torch.is_floating_point(v) else v) for k, v in sd.items()}
        self.s, self.mode = stage_idx, mode
        self.feats = [f.to(F64) for f in feats]
        self.proj = proj.to(F64)
        self.C, self.base, self.dtype = feats[0].shape[1], 8, F64
        self.p = "cost_regularization.%d." % stage_idx

    def warp_aggregate(self, feats, proj, hyps, rt=None, layout=None):
        vol = O.aggregate(self.feats, self.proj, hyps, self.sd, self.s, self.mode, warp_impl="gather")
        return vol.permute(0, 2, 3, 4, 1).contiguous()

    def warp_aggregate_rows(self, feats, rt, hyps, h, y0, rows, out_y, out, layout=None):
        B, D, R, w = hyps.shape
        full = hyps[:, :, out_y:out_y + 1].expand(B, D, h, w).clone()  # rows outside the window: any depth
        full[:, :, y0:y0 + rows] = hyps[:, :, out_y:out_y + rows]
        out[:, :, out_y:out_y + rows] = self.warp_aggregate(feats, None, full)[:, :, y0:y0 + rows]
        return out

    def unet_buffers(self, B, D, h, w):
        b = self.base
        spec = ((0, b), (1, 2 * b), (1, 2 * b), (2, 4 * b), (2, 4 * b), (3, 8 * b), (3, 8 * b))
        return [torch.empty(B, D >> l, h >> l, w >> l, c, dtype=F64) for l, c in spec]

    def unet_layer(self, layer, D, h, w, inp, out):
        p = self.p + LAYERS[layer]
        x = inp.permute(0, 4, 1, 2, 3)
        if layer < 7:
            y = F.conv3d(x, self.sd[p + ".conv.weight"], stride=2 if layer in (1, 3, 5) else 1, padding=1)
        else:
            y = F.conv_transpose3d(x, self.sd[p + ".conv.weight"], stride=2, padding=1, output_padding=1)
        y = F.relu(O._bn(y, self.sd, p + ".bn"))
        if layer >= 7:
            y = y + out.permute(0, 4, 1, 2, 3)
        out.copy_(y.permute(0, 2, 3, 4, 1))
        return out

    def regress_c0(self, c0, hyps, prob_init=None, want_prob=True, scratch=None):
        logits = F.conv3d(c0.permute(0, 4, 1, 2, 3), self.sd[self.p + "prob.weight"], padding=1)[:, 0]
        o = O.regression(logits, hyps.to(F64))
        return o["depth"], o["photometric_confidence"], o["variance"], o["prob_volume"] if want_prob else None


def _case(H=40, W=24, D=8, N=3, s=2, B=1, mode="adaptive"):
    C = (32, 16, 8)[s]
    sd = model_state("depthnet_cfgA_" + mode)
    feats, P, hyps = depthnet_inputs(B=B, N=N, H=H, W=W, D=D, stage_idx=s, C=C)
    return sd, feats, P, hyps.to(F64), s, mode


def _unsharded(sd, feats, P, hyps, s, mode):
    sd64 = {k: (v.to(F64) if torch.is_floating_point(v) else v) for k, v in sd.items()}
    with torch.no_grad():
        return O.depthnet_stage(s, [f.to(F64) for f in feats], P.to(F64), hyps, sd64, mode, warp_impl="gather")


def _run_sharded(comm, case, warp):
    sd, feats, P, hyps, s, mode = case
    eng = CpuStageEngine(sd, s, mode, feats, P)
    H, W = hyps.shape[2:]
    with torch.no_grad():
        return S.sharded_stage(comm, eng, None, None, None, hyps, H, W, warp=warp)


def _compare(got, ref):
    depth, conf, var, prob = got
    np.testing.assert_allclose(depth.numpy(), ref["depth"].numpy(), rtol=1e-10)
    np.testing.assert_allclose(prob.numpy(), ref["prob_volume"].numpy(), rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(var.numpy(), ref["variance"].numpy(), rtol=1e-8)
    np.testing.assert_allclose(conf.numpy(), ref["photometric_confidence"].numpy(), rtol=1e-9)


def test_slab_and_plane_partitions():
    assert S.slab_rows(296, 8) == [0, 40, 80, 120, 160, 200, 232, 264, 296]  # cfgD stage 1 over 8 GPUs
    for h, P in ((1184, 8), (592, 8), (264, 8), (40, 3), (16, 2), (8, 1)):
        ys = S.slab_rows(h, P)
        assert ys[0] == 0 and ys[-1] == h and all((b - a) % 8 == 0 and b - a >= 8 for a, b in zip(ys, ys[1:]))
    with pytest.raises(ValueError):
        S.slab_rows(56, 8)  # 7 level-3 rows for 8 ranks
    for D, P in ((64, 8), (32, 8), (8, 8), (8, 3), (4, 8)):
        ds = S.depth_planes(D, P)
        assert ds[0] == 0 and ds[-1] == D and all(0 <= b - a <= -(-D // P) for a, b in zip(ds, ds[1:]))


@pytest.mark.parametrize("P", [1, 2, 3, 5])
@pytest.mark.parametrize("warp", ["depth", "rows", "gather"])
def test_thread_group_matches_unsharded(P, warp):
    case = _case()
    ref = _unsharded(*case)
    for got in S.ThreadGroup(P).run(lambda comm: _run_sharded(comm, case, warp)):
        _compare(got, ref)


def test_thread_group_variance_batch2_stage1():
    """variance aggregation, B = 2 with distinct samples, C = 32 / D = 16 (stage-1 channel count), P = 2."""
    sd, feats, P, hyps, s, mode = _case(H=32, W=24, D=16, N=3, s=0, B=2, mode="variance")
    hyps[1] *= 1.03
    case = (sd, feats, P, hyps, s, mode)
    ref = _unsharded(*case)
    for got in S.ThreadGroup(2).run(lambda comm: _run_sharded(comm, case, "depth")):
        _compare(got, ref)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gloo_worker(rank, world, port, warp, q, B=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        case = _case(B=B)
        if B > 1:
            case[3][1] *= 1.03  # distinct samples
        got = _run_sharded(S.TorchComm(), case, warp)
        if rank == world - 1:
            ref = _unsharded(*case)
            try:
                _compare(got, ref)
                q.put(("ok", None))
            except AssertionError as e:
                q.put(("fail", str(e)))
    finally:
        dist.destroy_process_group()


def _cascade_case():
    """A whole cascade (FeatureNet, GeoFeatureFusion, three stages 48/32/8) at 96 x 64, 3 views, float64."""
    from common import forward_inputs
    sd = model_state("forward_cfgB_640x512")
    sd = {k: (v.to(F64) if torch.is_floating_point(v) else v) for k, v in sd.items()}
    imgs, proj, dv, _ = forward_inputs(1, 3, 64, 96)
    return sd, imgs.to(F64), {k: v.to(F64) for k, v in proj.items()}, dv.to(F64)


def _cascade(sd, imgs, proj, dv, comm=None, warp="depth"):
    """oracle.cascade_forward with every stage's DepthNet depth-sharded over ``comm`` (None: unsharded)."""
    def stage(s, fs, P, hyps):
        eng = CpuStageEngine(sd, s, "adaptive", fs, P)
        d, c, v, p = S.sharded_stage(comm, eng, None, None, None, hyps.to(F64), hyps.shape[2], hyps.shape[3], warp=warp)
        return {"depth": d, "photometric_confidence": c, "variance": v, "prob_volume": p, "depth_values": hyps}
    with torch.no_grad():
        return O.cascade_forward(sd, imgs, proj, dv, (48, 32, 8), "adaptive", warp_impl="gather",
                                 depthnet=None if comm is None else stage)


def _gloo_cascade_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        case = _cascade_case()
        got = _cascade(*case, comm=S.TorchComm())
        if rank == world - 1:
            ref = _cascade(*case)
            try:
                for st in ("stage1", "stage2", "stage3"):
                    # float64: the sharded U-Net's CPU GEMM blocking differs with the slab height, and the cascade
                    # re-centres each stage on the previous depth, so summation-order noise grows stage by stage
                    np.testing.assert_allclose(got[st]["depth"].numpy(), ref[st]["depth"].numpy(), rtol=1e-9)
                    np.testing.assert_allclose(got[st]["prob_volume"].numpy(), ref[st]["prob_volume"].numpy(),
                                               rtol=1e-7, atol=1e-10)
                q.put(("ok", None))
            except AssertionError as e:
                q.put(("fail", str(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_whole_cascade_every_stage_sharded():
    """The whole cascade (front-end replicated, every stage's DepthNet depth-sharded over 2 gloo ranks) against the
    unsharded float64 cascade: the all-to-all, halo exchanges and all-gather of all three stages, and the next
    stage's hypotheses and GeoFeatureFusion reading the gathered maps."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_cascade_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(280)
        assert p.exitcode == 0
    status, msg = q.get(timeout=10)
    assert status == "ok", msg


@pytest.mark.timeout(180)
@pytest.mark.parametrize("world,warp,B", [(2, "depth", 1), (3, "depth", 1), (3, "rows", 1), (2, "depth", 2),
                                                (3, "gather", 2)])
def test_gloo_world_matches_unsharded(world, warp, B):
    """Real torch.distributed P2P (gloo, one process per rank): all-to-all, halo exchange, all-gather. B = 2 runs the
    U-Net as two batch halves with each half's halo transfer outstanding while the other half computes."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, warp, q, B)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(150)
        assert p.exitcode == 0
    status, msg = q.get(timeout=10)
    assert status == "ok", msg
