"""GPU: no kernel writes outside the tensors it is given.

Every output (U-Net level tensors, the warp's volume, the stage workspace and the stage's depth / confidence /
variance / probability outputs) is placed inside a larger buffer whose head and tail hold a byte pattern; after the
launch both guard bands must be intact. A write past a tensor's end lands in whatever the caching allocator put
next to it -- in the concurrent-stream forward that can be another sub-batch's live tensor -- and the parity tests,
which compare only the tensors themselves, cannot see it.
"""
import ctypes

import pytest
import torch

from common import model_state

pytestmark = pytest.mark.gpu
DEV = "cuda"
GUARD = 1 << 16  # bytes before and after each output
PATTERN = 0x5A


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from damvsnet_amd import _capi
    _capi.load_library()


class Guarded:
    """A tensor of `shape` / `dtype` inside a guard-banded byte buffer."""

    def __init__(self, shape, dtype, init=None):
        n = torch.empty((), dtype=dtype).element_size()
        for d in shape:
            n *= d
        self.n = n
        self.buf = torch.full((GUARD + n + GUARD,), PATTERN, dtype=torch.uint8, device=DEV)
        self.t = self.buf[GUARD:GUARD + n].view(dtype).view(*shape)
        if init is not None:
            self.t.copy_(init)

    def check(self, what):
        torch.cuda.synchronize()
        head = self.buf[:GUARD] != PATTERN
        tail = self.buf[GUARD + self.n:] != PATTERN
        assert not bool(head.any()), "%s: %d bytes written before the tensor (nearest at -%d)" % (
            what, int(head.sum()), GUARD - int(head.nonzero().max()))
        assert not bool(tail.any()), "%s: %d bytes written past the end (first at +%d)" % (
            what, int(tail.sum()), int(tail.nonzero().min()))


# (stage index, C, D, h, w): the three stages at cfgC's channel widths and depths, at sizes that are multiples of 8
# but not of the kernels' tile sizes, and at
# stage 2's full cfgC size (the layer shapes of the concurrent-stream test)
CASES = [(0, 32, 48, 40, 72), (1, 16, 32, 56, 88), (2, 8, 8, 24, 104), (1, 16, 32, 592, 800)]
SRC = (None, 0, 1, 2, 3, 4, 5, 6, 4, 2)
DST = (0, 1, 2, 3, 4, 5, 6, 4, 2, 0)


def _net(dtype):
    from damvsnet_amd.cascade import CascadeMVSNet
    net = CascadeMVSNet(ndepths=[48, 32, 8], compute_dtype=dtype)
    net.load_state_dict(model_state("depthnet_cfgA_adaptive"), strict=True)
    return net.to(DEV).eval()


def _inputs(s, C, D, h, w, B, N, dtype):
    from damvsnet_amd import synth
    from damvsnet_amd.engine import hypotheses
    H, W = h * (4 >> s), w * (4 >> s)
    proj, _, dv = synth.cameras(B, N, H, W)
    P = torch.from_numpy(proj["stage%d" % (s + 1)]).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(s)
    if s == 0:
        hyps = hypotheses(torch.from_numpy(dv).to(DEV), D, H, W, 4)
    else:
        pd = 600 + 100 * torch.rand(B, H // 4, W // 4, device=DEV, generator=g)
        pv = 5 + 20 * torch.rand(B, H // 4, W // 4, device=DEV, generator=g)
        hyps = hypotheses(torch.from_numpy(dv).to(DEV), D, H, W, 4 >> s, pd, pv)
    feats = [torch.randn(B, h, w, C, generator=g, device=DEV).to(dtype) for _ in range(N)]
    return P, hyps, feats


@pytest.mark.timeout(240)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32], ids=["bf16", "f32"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "s%d_%dx%d" % (c[0], c[3], c[4]))
def test_unet_layers_and_warp_write_inside_their_outputs(case, dtype):
    s, C, D, h, w = case
    B, N = 2, 5
    net = _net(dtype)
    eng = net.DepthNet.engine(s, net.cost_regularization[s], torch.device(DEV))
    P, hyps, feats = _inputs(s, C, D, h, w, B, N, dtype)
    with torch.no_grad():
        vol = Guarded((B, D, h, w, C), dtype)
        eng.warp_aggregate(feats, P, hyps, out=vol.t)
        vol.check("warp_aggregate NHWC")
        from damvsnet_amd import _capi
        from damvsnet_amd.engine import block_channels
        volb = Guarded((B, D, h, w, C), dtype)
        eng.warp_aggregate(block_channels(feats), P, hyps, layout=_capi.DAMVS_LAYOUT_CBLOCK, out=volb.t)
        volb.check("warp_aggregate channel-blocked")
        bufs = eng.unet_buffers(B, D, h, w)
        g = torch.Generator(device=DEV).manual_seed(1)
        for b in bufs:  # the deconvs add into their outputs: start from finite values
            b.copy_(torch.randn(b.shape, generator=g, device=DEV).to(dtype))
        for layer in range(10):
            src = vol.t if layer == 0 else bufs[SRC[layer]]
            dst = Guarded(bufs[DST[layer]].shape, dtype, init=bufs[DST[layer]])
            eng.unet_layer(layer, D, h, w, src, dst.t)
            dst.check("U-Net layer %d" % layer)
            bufs[DST[layer]] = dst.t


@pytest.mark.timeout(240)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32], ids=["bf16", "f32"])
@pytest.mark.parametrize("case", CASES[:3], ids=lambda c: "s%d_%dx%d" % (c[0], c[3], c[4]))
def test_stage_forward_writes_inside_workspace_and_outputs(case, dtype):
    from damvsnet_amd import _capi
    s, C, D, h, w = case
    B, N = 2, 5
    net = _net(dtype)
    eng = net.DepthNet.engine(s, net.cost_regularization[s], torch.device(DEV))
    P, hyps, feats = _inputs(s, C, D, h, w, B, N, dtype)
    lib = _capi.load_library()
    n = ctypes.c_size_t()
    assert lib.damvs_stage_workspace_size(eng.handle, B, N, D, h, w, ctypes.byref(n)) == 0
    ws = Guarded((n.value,), torch.uint8)
    outs = {k: Guarded((B, h, w), torch.float32) for k in ("depth", "conf", "var")}
    prob = Guarded((B, D, h, w), torch.float32)
    fptrs = (ctypes.c_void_p * N)(*[f.data_ptr() for f in feats])
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    with torch.no_grad():
        for prob_init in (None, torch.rand(B, D, h, w, device=DEV)):
            rc = lib.damvs_stage_forward(eng.handle, _capi.stream_ptr(torch.device(DEV)), B, N, D, h, w, fptrs, p(P),
                                         p(hyps), p(prob_init) if prob_init is not None else None, p(ws.t), ws.n,
                                         p(outs["depth"].t), p(outs["conf"].t), p(outs["var"].t), p(prob.t))
            _capi.check(rc)
            ws.check("stage workspace")
            for k, o in outs.items():
                o.check(k)
            prob.check("prob_volume")
