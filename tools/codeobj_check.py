"""Code-object audit of the built library: per kernel, VGPRs, AGPRs, LDS, scratch (private segment) and spills,
read from the gfx950 code objects' metadata notes (llvm-readelf --notes) inside libdamvs.so's .hip_fatbin.

  python tools/codeobj_check.py [lib] [--all]

Prints the kernels that use scratch or spill VGPRs (all kernels with --all; SGPR spills go to VGPR lanes, not
memory, and are listed but not counted). tests/test_codeobj.py keeps that list to the
allowed entries: a register array or lambda closure that hipcc leaves in scratch costs 2-7x on the hot kernels
(conv2d_wide_kernel<float> at input stride 2, round 4).
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib):
    """The gfx950 ELF code objects of every offload bundle in lib's .hip_fatbin section."""
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", ".hip_fatbin=" + fat, lib, os.devnull],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
    out, pos = [], data.find(MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", data, pos + 24)
        q = pos + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, q)
            triple = data[q + 24:q + 24 + tl].decode()
            q += 24 + tl
            if "gfx950" in triple and size:
                out.append(data[pos + off:pos + off + size])
        pos = data.find(MAGIC, pos + 24)
    return out


def kernels(lib):
    """{kernel symbol: {vgpr, agpr, lds, priv, spill}} over all code objects."""
    res = {}
    with tempfile.TemporaryDirectory() as td:
        for i, co in enumerate(code_objects(lib)):
            p = os.path.join(td, "co%d.o" % i)
            open(p, "wb").write(co)
            txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", p], check=True,
                                 capture_output=True, text=True).stdout
            for blk in re.split(r"\n\s+- \.agpr_count:", txt)[1:]:
                agpr = int(blk.split()[0])
                name = re.search(r"\.name:\s+(\S+)", blk).group(1)

                def g(k):
                    m = re.search(r"\." + k + r":\s+(\d+)", blk)
                    return int(m.group(1)) if m else 0
                res[name] = dict(vgpr=g("vgpr_count"), agpr=agpr, lds=g("group_segment_fixed_size"),
                                 priv=g("private_segment_fixed_size"), spill=g("vgpr_spill_count"),
                                 sspill=g("sgpr_spill_count"))
    return res


def demangled(names):
    try:
        r = subprocess.run([os.path.join(LLVM, "llvm-cxxfilt")], input="\n".join(names), capture_output=True,
                           text=True, check=True)
        return r.stdout.split("\n")
    except (OSError, subprocess.CalledProcessError):
        return list(names)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    lib = args[0] if args else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                            "damvsnet_amd", "libdamvs.so")
    ks = kernels(lib)
    names = sorted(ks)
    show = names if "--all" in sys.argv else [n for n in names if ks[n]["priv"] or ks[n]["spill"]]
    for n, d in zip(show, demangled(show)):
        k = ks[n]
        print("vgpr %3d agpr %3d lds %6d priv %4d vspill %3d sspill %3d  %s"
              % (k["vgpr"], k["agpr"], k["lds"], k["priv"], k["spill"], k["sspill"], d[:150]))
    print("%d kernels, %d with scratch or spills" % (len(ks), sum(1 for k in ks.values() if k["priv"] or k["spill"])))


if __name__ == "__main__":
    main()
