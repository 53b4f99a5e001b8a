"""GPU: kernels on concurrent HIP streams.

``CascadeMVSNet.forward(streams=S)`` runs the batch as S sub-batches on concurrent streams (bench.py's timed
steps, the bf16 headline and the fp32 parity path alike). Every kernel sees per sample the inputs it sees in one
batch, so all outputs must be bitwise the one-stream result, at both dtypes. The stage-2 warp launched beside U-Net layers on another stream must also reproduce its
solo output: until round 2 it staged its cameras in LDS, and beside a U-Net kernel that copy came back altered
(76 of 80 launches beside conv0, tools/streams_race_kernel.py); the cameras are now scalar loads.
"""
import numpy as np
import pytest
import torch

from common import model_state, forward_inputs

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from damvsnet_amd import _capi
    _capi.load_library()


def _perturb(P):
    """Per-sample cameras (synth broadcasts one): source translations x (1 + 0.15 b), a small extra yaw."""
    P = P.clone()
    for b in range(P.shape[0]):
        a = 0.01 * b
        R = torch.tensor([[np.cos(a), 0.0, np.sin(a)], [0.0, 1.0, 0.0], [-np.sin(a), 0.0, np.cos(a)]],
                         dtype=P.dtype)
        P[b, 1:, 0, :3, 3] *= 1.0 + 0.15 * b
        P[b, 1:, 0, :3, :3] = R @ P[b, 1:, 0, :3, :3]
    return P


# (dtype, stage, layout): the product's own warp kernel for each stage and dtype (layout None: the library's choice,
# damvs_warp_feat_blocked, as damvs_stage_forward makes it) -- bf16 stage 2 (2 lanes per voxel), stage 1 (4 lanes); fp32
# stage 2 (4 lanes), stage 1 (8 lanes: 128-byte pixels); plus the one-lane kernel on channel-blocked maps (bf16 stage 2)
# and stage 3 (full resolution, 8 channels: the one-lane kernel at bf16, 2 lanes at fp32 on the unrolled view loop the
# packed-FP32 fix brought back)
# and the N = 7 (cfgD) unrolled split kernels at stage 2
WARP_CASES = [(torch.bfloat16, 1, None, 5), (torch.bfloat16, 1, "cblock", 5), (torch.bfloat16, 0, None, 5),
              (torch.float32, 1, None, 5), (torch.float32, 0, None, 5), (torch.bfloat16, 2, None, 5),
              (torch.float32, 2, None, 5), (torch.bfloat16, 1, None, 7), (torch.float32, 1, None, 7),
              (torch.bfloat16, 0, None, 7), (torch.float32, 0, None, 7)]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("dtype,s,layout,N", WARP_CASES,
                         ids=["bf16-s2", "bf16-s2-cblock", "bf16-s1", "f32-s2", "f32-s1", "bf16-s3", "f32-s3",
                              "bf16-s2-n7", "f32-s2-n7", "bf16-s1-n7", "f32-s1-n7"])
def test_warp_beside_unet_layers_on_another_stream(dtype, s, layout, N):
    from damvsnet_amd.cascade import CascadeMVSNet
    from damvsnet_amd.engine import hypotheses, block_channels, proj_prepare, warp_blocked
    from damvsnet_amd import _capi, synth
    net = CascadeMVSNet(ndepths=[48, 32, 8], compute_dtype=dtype)
    net.load_state_dict(model_state("depthnet_cfgA_adaptive"), strict=True)
    net = net.to(DEV).eval()
    B, H, W = 2, 1184, 1600
    C, D, scale = {0: (32, 48, 4), 1: (16, 32, 2), 2: (8, 8, 1)}[s]
    h, w = H // scale, W // scale
    proj, _, dv = synth.cameras(B, N, H, W)
    P = _perturb(torch.from_numpy(proj["stage%d" % (s + 1)])).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(0)
    if s == 0:
        hyps = hypotheses(torch.from_numpy(dv).to(DEV), D, H, W, scale)
    else:  # refined per-pixel hypotheses from the previous stage's maps, as the pipeline has them
        pd = 600 + 100 * torch.rand(B, H // (2 * scale), W // (2 * scale), device=DEV, generator=g)
        pv = 5 + 20 * torch.rand(B, H // (2 * scale), W // (2 * scale), device=DEV, generator=g)
        hyps = hypotheses(torch.from_numpy(dv).to(DEV), D, H, W, scale, pd, pv)
    feats = [torch.randn(B, h, w, C, generator=g, device=DEV).to(dtype) for _ in range(N)]
    eng = net.DepthNet.engine(s, net.cost_regularization[s], torch.device(DEV))
    blocked = warp_blocked(C, feats[0].element_size(), N) if layout is None else layout == "cblock"
    with torch.no_grad():
        rt = proj_prepare(P)
        fb = block_channels(feats) if blocked else feats
        lay = _capi.DAMVS_LAYOUT_CBLOCK if blocked else _capi.DAMVS_LAYOUT_NHWC
        warp = lambda: eng.warp_aggregate(fb, None, hyps, rt=rt, layout=lay)  # noqa: E731
        vol = warp()
        bufs = eng.unet_buffers(B, D, h, w)
        torch.cuda.synchronize()
        ref = vol.clone()
        sa, sb, main = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.current_stream()
        for layer in (0, 1, 7):
            src = vol if layer == 0 else bufs[(None, 0, 1, 2, 3, 4, 5, 6, 4, 2)[layer]]
            dst = bufs[(0, 1, 2, 3, 4, 5, 6, 4, 2, 0)[layer]]
            for _ in range(3):
                sa.wait_stream(main)
                sb.wait_stream(main)
                with torch.cuda.stream(sa):
                    for _ in range(6):
                        eng.unet_layer(layer, D, h, w, src, dst)
                with torch.cuda.stream(sb):
                    outs = [warp() for _ in range(6)]
                torch.cuda.synchronize()
                bad = [int((o != ref).sum()) for o in outs]
                assert not any(bad), (layer, bad)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("streams,offset", [(2, None), (4, None), (2, "stage1.hypotheses"), (4, "stage2.geofusion")])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_forward_sub_batches_on_streams_bitwise(streams, offset, dtype):
    """Sub-batches on concurrent streams (optionally each starting when the previous one reaches ``offset``) give the
    one-stream forward's bits."""
    from damvsnet_amd.cascade import CascadeMVSNet
    net = CascadeMVSNet(ndepths=[48, 32, 8], compute_dtype=dtype,
                        frontend_dtype=torch.bfloat16 if dtype == torch.bfloat16 else None)
    net.load_state_dict(model_state("forward_cfgB_640x512"), strict=True)
    net = net.to(DEV).eval()
    imgs, proj, dv, ins = forward_inputs(4, 5, 512, 640)
    imgs, dv = imgs.to(DEV), dv.to(DEV)
    proj = {k: _perturb(v).to(DEV) for k, v in proj.items()}
    with torch.no_grad():
        ref = net(imgs, proj, dv)
        for _ in range(3):
            got = net(imgs, proj, dv, streams=streams, stream_offset=offset)
            torch.cuda.synchronize()
            for st in ("stage1", "stage2", "stage3"):
                for k in ("depth", "photometric_confidence", "variance", "prob_volume", "depth_values"):
                    assert torch.equal(got[st][k], ref[st][k]), (st, k)
            assert torch.equal(got["depth"], ref["depth"])
