"""Build libdamvs.so in-tree with hipcc for gfx950 (no CMake, no JIT cache).

``python -m damvsnet_amd.build`` or ``damvsnet_amd.build.build()``. Objects are compiled in
parallel and linked into ``damvsnet_amd/libdamvs.so``; a rebuild is skipped when the library
is newer than every source and header.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(REPO, "include")
LIB = os.path.join(PKG, "libdamvs.so")
OBJ = os.path.join(PKG, "build_obj")
ARCH = os.environ.get("DAMVS_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

CFLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-I" + INCLUDE, "-I" + CSRC,
          "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return any(os.path.getmtime(p) > t for p in deps)


def _compile(src):
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    lang = ["-x", "hip"] if src.endswith(".hip") else ["-x", "hip"]
    cmd = [HIPCC] + CFLAGS + lang + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s\n%s" % (src, " ".join(cmd), r.stderr))
    return obj, r.stderr


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    os.makedirs(OBJ, exist_ok=True)
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        results = list(ex.map(_compile, srcs))
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
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
