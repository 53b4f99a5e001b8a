"""Diagnostic builds of libdamvs.so with the bf16 in-place skip epilogue variants of k_conv3d.hip
(DAMVS_DIAG_SKIP_EPI = 1..4, see the macro's comment), for tools/diag_unet_repro.py A/B runs on the GPU box:

  python tools/diag_skip_epilogue.py            # here: builds damvsnet_amd/diag/libdamvs_skip{1..4}.so
  DAMVS_LIB=damvsnet_amd/diag/libdamvs_skip1.so DAMVS_DECONV_NO_ZSLIDE=1 python tools/diag_unet_repro.py ...

Only k_conv3d.hip is recompiled; the other objects come from the product build (damvsnet_amd/build_obj).
"""
import glob
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from damvsnet_amd import build as B  # noqa: E402


def main():
    B.build()
    out_dir = os.path.join(B.PKG, "diag")
    os.makedirs(out_dir, exist_ok=True)
    objs = [o for o in glob.glob(os.path.join(B.OBJ, "*.o")) if not o.endswith("k_conv3d.hip.o")]
    for v in (1, 2, 3, 4):
        obj = os.path.join(out_dir, "k_conv3d_skip%d.o" % v)
        subprocess.run([B.HIPCC] + B.CFLAGS + ["-DDAMVS_DIAG_SKIP_EPI=%d" % v, "-x", "hip", "-c",
                                               os.path.join(B.CSRC, "k_conv3d.hip"), "-o", obj], check=True)
        lib = os.path.join(out_dir, "libdamvs_skip%d.so" % v)
        subprocess.run([B.HIPCC, "-shared", "-fPIC", "--offload-arch=" + B.ARCH, "-o", lib, obj] + objs, check=True)
        print(lib)


if __name__ == "__main__":
    main()
