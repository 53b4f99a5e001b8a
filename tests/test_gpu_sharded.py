"""GPU: depth-sharded execution (damvsnet_amd/sharded.py) on one device against the unsharded HIP path.

P ranks are emulated as P threads on cuda:0 (sharded.ThreadGroup) running the real per-rank program: the
D-sharded (or row-windowed) warp through the C ABI, the all-to-all re-shard to H-slabs, the U-Net layer by
layer (damvs_costreg_layer) on haloed slabs with halo exchange after every layer, the local regression
(damvs_stage_regress) and the all-gather of the rows. Every voxel and every layer output is produced by the
same kernel arithmetic from the same inputs as in damvs_stage_forward, so the result must be BITWISE equal to
the unsharded stage (fp32 and bf16). A two-process run over torch.distributed (gloo, device tensors staged
through the host; both ranks on cuda:0) covers the TorchComm path.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from common import model_state, depthnet_inputs, forward_inputs

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from damvsnet_amd import _capi
    _capi.load_library()


def _stage_case(s, D, B, H, W, dtype, N=3):
    from damvsnet_amd.cascade import CascadeMVSNet
    C = (32, 16, 8)[s]
    net = CascadeMVSNet(ndepths=[48, 32, 8], compute_dtype=dtype)
    net.load_state_dict(model_state("depthnet_cfgA_adaptive"), strict=True)
    net = net.to(DEV).eval()
    feats, P, hyps = depthnet_inputs(B=B, N=N, H=H, W=W, D=D, stage_idx=s, C=C)
    for b in range(1, B):  # distinct samples
        hyps[b] *= 1.0 + 0.02 * b
    nhwc = [f.permute(0, 2, 3, 1).contiguous().to(DEV, dtype) for f in feats]
    return net, nhwc, P.to(DEV), hyps.to(DEV)


@pytest.mark.parametrize("warp", ["depth", "rows", "gather"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("s,D,B,H,W,P", [(1, 32, 2, 64, 80, 2), (1, 32, 1, 64, 80, 3), (2, 8, 2, 48, 56, 4),
                                         (0, 48, 1, 32, 48, 4)])
def test_sharded_stage_bitwise(s, D, B, H, W, P, dtype, warp):
    from damvsnet_amd.sharded import ThreadGroup, DepthShardedDepthNet
    net, nhwc, proj, hyps = _stage_case(s, D, B, H, W, dtype)
    cr = net.cost_regularization[s]
    with torch.no_grad():
        ref = net.DepthNet.forward_nhwc(s, nhwc, proj, hyps, cr)
        outs = ThreadGroup(P).run(lambda comm: DepthShardedDepthNet(net, comm, warp=warp)(s, nhwc, proj, hyps, cr))
    torch.cuda.synchronize()
    for r, o in enumerate(outs):
        for k in ("depth", "photometric_confidence", "variance", "prob_volume"):
            assert torch.equal(o[k], ref[k]), (r, k, (o[k] - ref[k]).abs().max().item())


@pytest.mark.parametrize("warp", ["depth", "gather"])
@pytest.mark.parametrize("s,D,H,W", [(0, 64, 296, 400), (1, 32, 592, 800), (2, 8, 1184, 1600)])
def test_sharded_stage_cfgD_8way_bitwise(s, D, H, W, warp):
    """BASELINE.json configs[3] (cfgD: DTU 1600x1184, 7 views, 64/32/8, bf16) at every stage's real size over 8
    emulated ranks, as bench.py --gpus 8 runs it: the H-slab mode ("depth": D-sharded warp -> all-to-all -> per-layer
    haloed U-Net -> row all-gather) and north_star's literal volume all-gather ("gather"), bitwise the unsharded
    stage on every rank."""
    from damvsnet_amd.sharded import ThreadGroup, DepthShardedDepthNet
    net, nhwc, proj, hyps = _stage_case(s, D, 1, H, W, torch.bfloat16, N=7)
    cr = net.cost_regularization[s]
    with torch.no_grad():
        ref = net.DepthNet.forward_nhwc(s, nhwc, proj, hyps, cr)
        outs = ThreadGroup(8).run(lambda comm: DepthShardedDepthNet(net, comm, warp=warp)(s, nhwc, proj, hyps, cr))
    torch.cuda.synchronize()
    assert len(outs) == 8
    for r, o in enumerate(outs):
        for k in ("depth", "photometric_confidence", "variance", "prob_volume"):
            assert torch.equal(o[k], ref[k]), (r, k, (o[k] - ref[k]).abs().max().item())


@pytest.mark.parametrize("warp", ["depth", "gather"])
@pytest.mark.parametrize("s,D,H,W", [(0, 64, 264, 480), (1, 32, 528, 960)])
def test_sharded_stage_cfgE_8way_bitwise(s, D, H, W, warp):
    """BASELINE.json configs[4] (cfgE: Tanks&Temples 1920x1056, 11 views, 64/32/8, bf16 on 8 GPUs) at stages 1-2's real
    sizes over 8 emulated ranks (stage 1: 264 rows = 33 groups of 8 over 8 slabs), both partitionings, bitwise the
    unsharded stage on every rank."""
    from damvsnet_amd.sharded import ThreadGroup, DepthShardedDepthNet
    net, nhwc, proj, hyps = _stage_case(s, D, 1, H, W, torch.bfloat16, N=11)
    cr = net.cost_regularization[s]
    with torch.no_grad():
        ref = net.DepthNet.forward_nhwc(s, nhwc, proj, hyps, cr)
        outs = ThreadGroup(8).run(lambda comm: DepthShardedDepthNet(net, comm, warp=warp)(s, nhwc, proj, hyps, cr))
    torch.cuda.synchronize()
    assert len(outs) == 8
    for r, o in enumerate(outs):
        for k in ("depth", "photometric_confidence", "variance", "prob_volume"):
            assert torch.equal(o[k], ref[k]), (r, k, (o[k] - ref[k]).abs().max().item())


def test_sharded_cascade_bitwise():
    """The whole cascade (160x128, 5 views, 48/32/8, bf16) with every stage's DepthNet over 4 emulated ranks
    (stage-1 slabs of 8 rows) equals the single-GPU forward bitwise at every stage."""
    from damvsnet_amd.cascade import CascadeMVSNet
    from damvsnet_amd.sharded import ThreadGroup, DepthShardedDepthNet
    net = CascadeMVSNet(ndepths=[48, 32, 8], compute_dtype=torch.bfloat16, frontend_dtype=torch.bfloat16)
    net.load_state_dict(model_state("forward_160x128_48_32_8"), strict=True)
    net = net.to(DEV).eval()
    imgs, proj, dv, ins = forward_inputs(1, 5, 128, 160)
    imgs, dv = imgs.to(DEV), dv.to(DEV)
    proj = {k: v.to(DEV) for k, v in proj.items()}
    with torch.no_grad():
        net(imgs, proj, dv)  # build the folded front-end once, outside the threads
        ref = net(imgs, proj, dv)
        outs = ThreadGroup(4).run(lambda comm: net(imgs, proj, dv, depthnet=DepthShardedDepthNet(net, comm)))
    torch.cuda.synchronize()
    for o in outs:
        for st in ("stage1", "stage2", "stage3"):
            for k in ("depth", "photometric_confidence", "variance", "prob_volume"):
                assert torch.equal(o[st][k], ref[st][k]), (st, k)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gloo_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from damvsnet_amd.sharded import TorchComm, DepthShardedDepthNet
        net, nhwc, proj, hyps = _stage_case(1, 32, 2, 64, 80, torch.bfloat16)
        cr = net.cost_regularization[1]
        with torch.no_grad():
            ref = net.DepthNet.forward_nhwc(1, nhwc, proj, hyps, cr)
            got = DepthShardedDepthNet(net, TorchComm())(1, nhwc, proj, hyps, cr)
        torch.cuda.synchronize()
        q.put((rank, all(torch.equal(got[k], ref[k]) for k in ("depth", "photometric_confidence", "variance",
                                                                "prob_volume"))))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_sharded_stage_two_processes_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(200)
        assert p.exitcode == 0
    res = dict(q.get(timeout=10) for _ in range(2))
    assert res == {0: True, 1: True}
