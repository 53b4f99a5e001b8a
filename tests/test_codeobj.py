"""Code-object hygiene of the built library (CPU: reads the gfx950 code objects' metadata, no GPU).

No kernel may use scratch memory or spill VGPRs, except proj_prepare_kernel (one thread per view: the 4x4 fp64
camera algebra, microseconds per step). A register array or a lambda closure that hipcc leaves in scratch turns a hot
kernel's LDS stores into flat stores and its operands into memory round trips: conv2d_wide_kernel<float> at input
stride 2 ran 5-7x its bf16 form until round 4 (tools/codeobj_check.py)."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

ALLOWED_SCRATCH = ("proj_prepare_kernel",)


def test_no_scratch_or_vgpr_spills():
    import codeobj_check as C
    lib = os.path.join(REPO, "damvsnet_amd", "libdamvs.so")
    if not os.path.exists(lib):
        pytest.skip("libdamvs.so not built")
    if not os.path.exists(os.path.join(C.LLVM, "llvm-readelf")):
        pytest.skip("no ROCm llvm tools")
    ks = C.kernels(lib)
    assert len(ks) > 100  # every translation unit's code object was found
    bad = sorted(n for n, k in ks.items() if (k["priv"] or k["spill"]) and not any(a in n for a in ALLOWED_SCRATCH))
    assert not bad, "kernels with scratch or VGPR spills: %s" % bad
