"""Build libdamvs.so in-tree with hipcc for gfx950 (no CMake, no JIT cache).

``python -m damvsnet_amd.build`` or ``damvsnet_amd.build.build()``. Objects are compiled in
parallel and linked into ``damvsnet_amd/libdamvs.so``. The library carries the sha256 of the sources,
headers and compiler flags it was built from (``damvs_build_id()``, passed as -DDAMVS_BUILD_ID); a rebuild
is skipped only when that stamp (kept beside the library in ``libdamvs.so.build_id``) equals the hash of the
tree, and ``_capi.load_library`` refuses an in-tree library whose embedded stamp differs from the sources
beside it. So the library that runs is provably the build of the sources that travel with it (file times
play no part: a snapshot copied to another machine keeps the check meaningful).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(REPO, "include")
LIB = os.path.join(PKG, "libdamvs.so")
STAMP = LIB + ".build_id"
OBJ = os.path.join(PKG, "build_obj")
ARCH = os.environ.get("DAMVS_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

CFLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-I" + INCLUDE, "-I" + CSRC,
          "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]

# Per-file extra flags. k_warp.hip is built without the SLP vectorizer so that its kernels carry no packed-FP32 VALU
# ops (v_pk_fma/mul/add_f32): with those, the warp kernels' lanes 48-63 computed wrong tap coordinates while MFMA
# kernels of another stream shared the CU (DESIGN.md §4 "Concurrent streams"; profiles/r05/diag_streams/r05w).
FILE_FLAGS = {"k_warp.hip": ["-fno-slp-vectorize"]}
# Round 6 widened the rule to every kernel without MFMA instructions that can share a CU with another stream's MFMA
# kernels (tests/test_isa_pins.py test_valu_kernels_carry_no_packed_fp32_ops): the plane-input conv2d layers
# (k_planes.hip), the hypotheses / GeoFF depth pyramid / camera algebra (k_geometry.hip), the VALU prob conv,
# regression, range check and magnitude kernels (k_regress.hip) and depth fusion (k_fusion.hip).
# Both vectorizers are off there: the loop vectorizer, too, emits packed-FP32 ops (grid-stride loops by two).
for _f in ("k_planes.hip", "k_geometry.hip", "k_regress.hip", "k_fusion.hip"):
    FILE_FLAGS[_f] = ["-fno-slp-vectorize", "-fno-vectorize"]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _inputs():
    return sources() + sorted(glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h")))


def source_hash(arch: str | None = None) -> str:
    """First 16 hex digits of sha256 over (path relative to the repo, contents) of every source and header, plus
    the compiler flags that do not depend on where the repo lives (``arch``: the offload arch to hash the flags for,
    default DAMVS_ARCH / gfx950)."""
    h = hashlib.sha256()
    for p in _inputs():
        h.update(os.path.relpath(p, REPO).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    flags = [f for f in CFLAGS if not f.startswith("-I")]
    if arch is not None:
        flags = ["--offload-arch=" + arch if f.startswith("--offload-arch=") else f for f in flags]
    h.update(" ".join(flags).encode())
    for name in sorted(FILE_FLAGS):
        h.update(("\0%s:%s" % (name, " ".join(FILE_FLAGS[name]))).encode())
    return h.hexdigest()[:16]


def stamp() -> str | None:
    try:
        with open(STAMP) as f:
            return f.read().strip()
    except OSError:
        return None


def _stale(want: str) -> bool:
    return not os.path.exists(LIB) or stamp() != want


def _compile(src, build_id):
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    cmd = [HIPCC] + CFLAGS + FILE_FLAGS.get(os.path.basename(src), []) + \
        ['-DDAMVS_BUILD_ID="%s"' % build_id, "-x", "hip", "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s\n%s" % (src, " ".join(cmd), r.stderr))
    return obj, r.stderr


def build(force: bool = False, verbose: bool = False) -> str:
    want = source_hash()
    if not force and not _stale(want):
        if verbose:
            print("libdamvs.so up to date: build id %s == sources %s" % (stamp(), want), file=sys.stderr)
        return LIB
    os.makedirs(OBJ, exist_ok=True)
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        results = list(ex.map(lambda s: _compile(s, want), srcs))
    objs = [o for o, _ in results]
    if verbose:
        for (_, err), s in zip(results, srcs):
            if err.strip():
                print("[%s]\n%s" % (os.path.basename(s), err), file=sys.stderr)
    tmp = LIB + ".tmp"
    cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", tmp] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n%s\n%s" % (" ".join(cmd), r.stderr))
    os.replace(tmp, LIB)
    with open(STAMP, "w") as f:
        f.write(want + "\n")
    if verbose:
        print("libdamvs.so built from sources %s" % want, file=sys.stderr)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
