"""Per-kernel gfx950 instruction text of the built library (llvm-objdump over the code objects in libdamvs.so).

  python tools/isa.py [--lib PATH] --list                   kernel symbols (demangled) with instruction counts
  python tools/isa.py [--lib PATH] --kernel SUBSTR [--out F] one kernel's instructions (addresses and encodings dropped)
  python tools/isa.py [--lib PATH] --hash SUBSTR             sha256 (16 hex) of each matching kernel's instruction text
  python tools/isa.py [--lib PATH] --mix SUBSTR              instruction-class counts of each matching kernel
  python tools/isa.py --update-pins --validated-by LOG       rewrite tests/isa_pins.json from the built library
                                                            (only after the GPU stream tests passed on this build:
                                                            LOG is the committed pytest log that shows it)

The instruction text is what tests/test_isa_pins.py hashes: branch targets are printed as offsets relative to the
kernel (so the text does not depend on where the linker placed the kernel) and nothing else of the object enters it.
"""
import argparse
import collections
import hashlib
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from codeobj_check import code_objects, LLVM  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "damvsnet_amd", "libdamvs.so")
PINS = os.path.join(REPO, "tests", "isa_pins.json")


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True,
                       check=True)
    return r.stdout.splitlines()


def disassemble(lib=LIB):
    """{mangled kernel symbol: [instruction text, ...]} over all gfx950 code objects of lib."""
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for i, co in enumerate(code_objects(lib)):
            p = os.path.join(td, "co%d.o" % i)
            with open(p, "wb") as f:
                f.write(co)
            txt = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn",
                                  "--no-leading-addr", "--mcpu=gfx950", p],
                                 check=True, capture_output=True, text=True).stdout
            cur, body = None, []
            for line in txt.splitlines():
                m = re.match(r"^(?:[0-9a-f]+\s+)?<(\S+)>:$", line.strip())
                if m:
                    if cur is not None:
                        out[cur] = body
                    cur, body = m.group(1), []
                    continue
                if cur is None:
                    continue
                t = line.split("//")[0].strip()
                if not t or t.startswith(";"):
                    continue
                # branch targets: "s_branch 123 <sym+0x40>" -> keep the relative label only
                t = re.sub(r"<[^>+]*\+(0x[0-9a-f]+)>", r"<+\1>", t)
                t = re.sub(r"\s+", " ", t)
                body.append(t)
            if cur is not None:
                out[cur] = body
    # only kernels (their symbols carry a .kd descriptor); drop helper labels with empty bodies
    return {k: v for k, v in out.items() if v and not k.endswith(".kd")}


def isa_hash(instrs):
    return hashlib.sha256("\n".join(instrs).encode()).hexdigest()[:16]


def hashes(lib=LIB):
    """{demangled kernel name: instruction-text hash} of every kernel in lib."""
    ks = disassemble(lib)
    names = sorted(ks)
    return {d: isa_hash(ks[k]) for k, d in zip(names, demangle(names))}


def compiler():
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--version"], capture_output=True, text=True)
    line = [l for l in r.stdout.splitlines() if "clang version" in l]
    return line[0].strip() if line else "unknown"


def classify(t):
    op = t.split()[0]
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=LIB)
    g = ap.add_mutually_exclusive_group(required=True)
    g.add_argument("--list", action="store_true")
    g.add_argument("--kernel")
    g.add_argument("--hash")
    g.add_argument("--mix")
    g.add_argument("--update-pins", action="store_true")
    ap.add_argument("--validated-by", default=None)
    ap.add_argument("--out")
    a = ap.parse_args()
    if a.update_pins:
        import json
        if not a.validated_by or not os.path.exists(os.path.join(REPO, a.validated_by)):
            sys.exit("--validated-by must name the committed GPU pytest log of tests/test_gpu_streams.py on this build")
        with open(PINS, "w") as f:
            json.dump({"compiler": compiler(), "validated_by": a.validated_by, "kernels": hashes(a.lib)}, f, indent=1,
                      sort_keys=True)
            f.write("\n")
        print("wrote", PINS)
        return
    ks = disassemble(a.lib)
    names = sorted(ks)
    dem = dict(zip(names, demangle(names)))
    sel = lambda s: [k for k in names if s in dem[k] or s in k]  # noqa: E731
    if a.list:
        for k in names:
            print("%6d  %s" % (len(ks[k]), dem[k]))
    elif a.kernel:
        m = sel(a.kernel)
        if not m:
            sys.exit("no kernel matches %r" % a.kernel)
        text = "".join("; %s\n%s\n" % (dem[k], "\n".join(ks[k])) for k in m)
        if a.out:
            with open(a.out, "w") as f:
                f.write(text)
        else:
            sys.stdout.write(text)
    elif a.hash:
        for k in sel(a.hash):
            print(isa_hash(ks[k]), dem[k])
    else:
        for k in sel(a.mix):
            c = collections.Counter(classify(t) for t in ks[k])
            print(dem[k])
            print("   " + "  ".join("%s %d" % kv for kv in sorted(c.items())))


if __name__ == "__main__":
    main()
