"""ctypes binding of libdamvs.so (include/damvs.h).

The library is loaded from the package directory only (built in-tree by
``damvsnet_amd.build``); there is no fallback: if it is missing or fails to load, every
product entry point raises. ``torch`` is imported first so that the HIP runtime PyTorch
already mapped (soname libamdhip64.so.7) is the one the library binds to.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the library load: shared HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DAMVS_LIB") or os.path.join(_HERE, "libdamvs.so")  # DAMVS_LIB: A/B builds in tools

DAMVS_F32, DAMVS_BF16 = 0, 1
DAMVS_AGG_ADAPTIVE, DAMVS_AGG_VARIANCE = 0, 1
DAMVS_LAYOUT_NHWC, DAMVS_LAYOUT_CBLOCK = 0, 1
ERRORS = {-1: "DAMVS_E_ARG", -2: "DAMVS_E_SHAPE", -3: "DAMVS_E_DTYPE", -4: "DAMVS_E_HIP", -5: "DAMVS_E_NOMEM",
          -6: "DAMVS_E_WORKSPACE", -7: "DAMVS_E_RANGE"}
DAMVS_E_RANGE = -7

c_int, c_float, c_size_t, c_void_p = ctypes.c_int, ctypes.c_float, ctypes.c_size_t, ctypes.c_void_p


class DamvsBN(ctypes.Structure):
    _fields_ = [("weight", c_void_p), ("bias", c_void_p), ("running_mean", c_void_p), ("running_var", c_void_p),
                ("eps", c_float)]


class DamvsCostregParams(ctypes.Structure):
    _fields_ = [("in_channels", c_int), ("base_channels", c_int), ("conv_weight", c_void_p * 10), ("bn", DamvsBN * 10),
                ("prob_weight", c_void_p)]


class DamvsAggweightParams(ctypes.Structure):
    _fields_ = [("in_channels", c_int), ("w1", c_void_p), ("bn1", DamvsBN), ("w2", c_void_p), ("bn2", DamvsBN)]


class DamvsConv2dDesc(ctypes.Structure):
    _fields_ = [("transposed", c_int), ("kernel", c_int), ("stride", c_int), ("padding", c_int),
                ("output_padding", c_int), ("cin", c_int), ("cout", c_int), ("c0", c_int), ("c0_at", c_int),
                ("c1", c_int), ("c1_at", c_int), ("ngeo", c_int), ("geo_at", c_int * 4), ("relu", c_int)]


FUSION_MAX_SRC = 10
_f = ctypes.c_float


class DamvsFusionCams(ctypes.Structure):
    _fields_ = [("kinv_ref", _f * 9), ("k_ref", _f * 9), ("einv_ref", _f * 16),
                ("t_sr", (_f * 16) * FUSION_MAX_SRC), ("k_src", (_f * 9) * FUSION_MAX_SRC),
                ("kinv_src", (_f * 9) * FUSION_MAX_SRC), ("t_rs", (_f * 16) * FUSION_MAX_SRC)]


# (name, restype, argtypes) — the full exported surface of include/damvs.h
SIGNATURES = (
    ("damvs_abi_version", c_int, ()),
    ("damvs_last_error_string", ctypes.c_char_p, ()),
    ("damvs_build_id", ctypes.c_char_p, ()),
    ("damvs_stage_create", c_int, (ctypes.POINTER(DamvsCostregParams), ctypes.POINTER(DamvsAggweightParams), c_int,
                                   c_int, ctypes.POINTER(c_void_p))),
    ("damvs_stage_destroy", c_int, (c_void_p,)),
    ("damvs_stage_workspace_size", c_int, (c_void_p, c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(c_size_t))),
    ("damvs_stage_forward", c_int, (c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(c_void_p),
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p,
                                    c_void_p)),
    ("damvs_stage_forward_probed", c_int, (c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                           ctypes.POINTER(c_void_p), c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                           c_void_p, c_void_p, c_void_p, c_void_p, ctypes.POINTER(c_void_p))),
    ("damvs_stage_status", c_int, (c_void_p, c_void_p, c_void_p, c_size_t)),
    ("damvs_proj_prepare", c_int, (c_void_p, c_int, c_int, c_void_p, c_void_p)),
    ("damvs_homo_warp", c_int, (c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                c_void_p)),
    ("damvs_warp_aggregate", c_int, (c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(c_void_p),
                                     c_int, c_void_p, c_void_p, c_void_p)),
    ("damvs_warp_feat_blocked", c_int, (c_int, c_int)),
    ("damvs_warp_feat_blocked_n", c_int, (c_int, c_int, c_int)),
    ("damvs_block_channels", c_int, (c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(c_void_p),
                                     ctypes.POINTER(c_void_p))),
    ("damvs_costreg_logits", c_int, (c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_size_t,
                                     c_void_p)),
    ("damvs_warp_aggregate_rows", c_int, (c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                          c_int, ctypes.POINTER(c_void_p), c_int, c_void_p, c_void_p, c_void_p)),
    ("damvs_costreg_layer", c_int, (c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p)),
    ("damvs_costreg_layer_scaled", c_int, (c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                           c_void_p, c_void_p)),
    ("damvs_tensor_amax", c_int, (c_void_p, c_void_p, ctypes.c_longlong, c_void_p)),
    ("damvs_stage_regress", c_int, (c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p)),
    ("damvs_regress", c_int, (c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                              c_void_p, c_void_p)),
    ("damvs_hypotheses", c_int, (c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p,
                                 c_int, c_int, c_void_p)),
    ("damvs_sparse_depth_pyramid", c_int, (c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_void_p, c_void_p)),
    ("damvs_fpn_top_forward", c_int, (c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p)),
    ("damvs_fpn_top_forward_f32", c_int, (c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                          ctypes.c_float, c_void_p, c_void_p)),
    ("damvs_conv2d_create", c_int, (ctypes.POINTER(DamvsConv2dDesc), c_void_p, c_void_p, c_int,
                                    ctypes.POINTER(c_void_p))),
    ("damvs_conv2d_destroy", c_int, (c_void_p,)),
    ("damvs_conv2d_out_size", c_int, (c_void_p, c_int, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                                      ctypes.POINTER(c_int))),
    ("damvs_conv2d_forward", c_int, (c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                     ctypes.POINTER(c_void_p), ctypes.POINTER(ctypes.c_longlong), c_void_p, c_void_p,
                                     c_int, c_void_p)),
    ("damvs_fusion_view", c_int, (c_void_p, c_int, c_int, c_int, c_void_p, ctypes.POINTER(c_void_p),
                                  ctypes.POINTER(c_void_p), ctypes.POINTER(ctypes.c_float), ctypes.POINTER(DamvsFusionCams),
                                  ctypes.c_double, ctypes.c_double, c_void_p, c_void_p, c_void_p)),
    ("damvs_conv2d_border_bias", c_int, (c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                         ctypes.POINTER(ctypes.c_float), c_void_p)),
)

_lib = None


class DamvsError(RuntimeError):
    def __init__(self, rc, msg):
        super().__init__("%s (%d): %s" % (ERRORS.get(rc, "DAMVS_E_?"), rc, msg))
        self.rc = rc


class DamvsRangeError(DamvsError, FloatingPointError):
    """DAMVS_E_RANGE: a stage forward produced non-finite depth / confidence / variance (damvs_stage_status)."""


def load_library(path: str = LIB_PATH):
    """Load and type the HIP library; raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError("libdamvs.so not found at %s — build it with `python -m damvsnet_amd.build` "
                           "(the product has no CPU/eager fallback)" % path)
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    ab = os.path.abspath(path) != os.path.abspath(os.path.join(_HERE, "libdamvs.so"))
    for name, res, args in SIGNATURES:
        if ab and not hasattr(lib, name):  # an A/B build of an older commit may lack later entry points
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = list(args)
    if lib.damvs_abi_version() != 1:
        raise RuntimeError("libdamvs ABI mismatch")
    if os.path.abspath(path) == os.path.abspath(os.path.join(_HERE, "libdamvs.so")):
        # the in-tree library must be the build of the sources beside it (A/B builds through DAMVS_LIB are exempt)
        from .build import source_hash, ARCH
        got, want = lib.damvs_build_id().decode(), source_hash()
        if got != want:
            other = [a for a in ("gfx950",) if a != ARCH and source_hash(a) == got]
            if other:
                raise RuntimeError("libdamvs.so was built from these sources for --offload-arch=%s, but DAMVS_ARCH=%s "
                                   "in this environment: unset it or rebuild" % (other[0], ARCH))
            raise RuntimeError("libdamvs.so is stale: built from sources %s, the tree holds %s (arch %s) — rebuild "
                               "with `python -m damvsnet_amd.build`" % (got, want, ARCH))
    _lib = lib
    return lib


def check(rc: int):
    if rc != 0:
        msg = _lib.damvs_last_error_string().decode(errors="replace")
        raise (DamvsRangeError if rc == DAMVS_E_RANGE else DamvsError)(rc, msg)


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def float_ptr(t):
    """ctypes float* into a contiguous host fp32 tensor (kept alive by the caller)."""
    assert t.device.type == "cpu" and t.dtype == torch.float32 and t.is_contiguous()
    return ctypes.cast(t.data_ptr(), ctypes.POINTER(ctypes.c_float))


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
