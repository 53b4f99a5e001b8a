"""CPU: the drop-in boundary — C-ABI library loads and exports every declared symbol; the Python
modules mirror the reference's constructor, state_dict keys and error behaviour. No compute call
is made (there is no GPU here)."""
import ctypes
import os
import re

import pytest
import torch

from conftest import REPO
from common import reference_keys, model_state

HEADER = os.path.join(REPO, "include", "damvs.h")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(damvs_\w+)\s*\(", src, flags=re.M)))


def test_library_builds_and_exports_every_symbol():
    from damvsnet_amd import build
    lib_path = build.build()
    lib = ctypes.CDLL(lib_path)
    syms = declared_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(lib, s), s
    assert lib.damvs_abi_version() == 1


def test_library_is_the_build_of_this_tree():
    """The in-tree library embeds the hash of the sources it was compiled from; it must be this tree's."""
    from damvsnet_amd import build, _capi
    build.build()
    lib = _capi.load_library()  # raises on a stale library
    assert lib.damvs_build_id().decode() == build.source_hash() == build.stamp()


def test_binding_covers_header():
    from damvsnet_amd import _capi
    bound = {name for name, _, _ in _capi.SIGNATURES}
    assert bound == set(declared_symbols())


def test_arg_errors_without_gpu():
    """Argument validation happens before any device work and reports through the error string."""
    from damvsnet_amd import _capi
    lib = _capi.load_library()
    rc = lib.damvs_proj_prepare(None, 1, 2, None, None)
    assert rc == -1 and b"null" in lib.damvs_last_error_string()
    rc = lib.damvs_hypotheses(None, 1, 8, 33, 40, 2, None, 0, None, None, 0, 0, ctypes.c_void_p(16))
    assert rc == -2
    rc = lib.damvs_stage_create(None, None, 0, 0, ctypes.byref(ctypes.c_void_p()))
    assert rc == -1


@pytest.mark.parametrize("arch", ["fpn", "unet"])
def test_state_dict_keys_match_reference(arch):
    from damvsnet_amd.cascade import CascadeMVSNet
    ref = reference_keys(arch)
    mine = {k: list(v.shape) for k, v in CascadeMVSNet(arch_mode=arch).state_dict().items()}
    assert mine == ref


def test_reference_state_dict_loads_strict():
    from damvsnet_amd.cascade import CascadeMVSNet
    net = CascadeMVSNet(ndepths=[48, 32, 8])
    net.load_state_dict(model_state("forward_160x128_48_32_8"), strict=True)


def test_ctor_defaults_mirror_reference():
    from damvsnet_amd.cascade import CascadeMVSNet
    net = CascadeMVSNet()
    assert net.ndepths == [64, 32, 8] and net.depth_interals_ratio == [4, 2, 1]
    assert net.DepthNet.mode == "adaptive" and net.grad_method == "detach"
    assert net.feature.out_channels == [32, 16, 8]


def test_cpu_inputs_fail_loudly():
    """The product path has no CPU fallback."""
    from damvsnet_amd.cascade import CascadeMVSNet
    net = CascadeMVSNet(ndepths=[48, 32, 8]).eval()
    with pytest.raises(ValueError, match="GPU"):
        net(torch.zeros(1, 3, 3, 64, 64), {}, torch.zeros(1, 192))
    from damvsnet_amd.depthnet import homo_warping
    with pytest.raises(ValueError, match="HIP device"):
        homo_warping(torch.zeros(1, 8, 8, 8), torch.eye(4)[None], torch.eye(4)[None], torch.ones(1, 2))


def test_warp_feature_layout_by_view_count():
    """damvs_warp_feat_blocked_n (host logic, no device work): NHWC in place wherever the channel-split warp takes the
    pixel (32 / 64 / 128 bytes at odd N >= 3), channel-blocked for wider pixels the one-lane warp gathers (even N:
    profiles/r05/ab_warp_layout_r05p.txt), NHWC for 16-byte pixels; the N-less entry point answers for N = 5."""
    from damvsnet_amd import _capi
    lib = _capi.load_library()
    F32, BF16 = _capi.DAMVS_F32, _capi.DAMVS_BF16
    for dt, C in ((F32, 32), (F32, 16), (BF16, 32)):  # 128 / 64 / 64-byte pixels
        assert lib.damvs_warp_feat_blocked_n(dt, C, 5) == 0 and lib.damvs_warp_feat_blocked_n(dt, C, 11) == 0
        assert lib.damvs_warp_feat_blocked_n(dt, C, 4) == 1 and lib.damvs_warp_feat_blocked_n(dt, C, 2) == 1
        assert lib.damvs_warp_feat_blocked(dt, C) == 0
    for dt, C in ((F32, 8), (BF16, 16), (BF16, 8)):  # 32 / 32 / 16-byte pixels: never blocked
        for n in (2, 4, 5):
            assert lib.damvs_warp_feat_blocked_n(dt, C, n) == 0
    assert lib.damvs_warp_feat_blocked_n(F32, 24, 5) == 1  # 96-byte pixels: no split form
    assert lib.damvs_warp_feat_blocked_n(F32, 32, 1) < 0 and lib.damvs_warp_feat_blocked_n(7, 32, 5) < 0

