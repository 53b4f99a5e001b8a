"""Register / occupancy table of libdamvs kernels from hipcc's kernel-resource-usage remarks.

  python tools/kres.py k_conv3d [k_conv2d ...] [--grep PATTERN]

Compiles each csrc/<unit>.hip for gfx950 (the library's flags) and prints one line per kernel instance:
VGPRs, AGPRs, spills, LDS bytes and waves per SIMD, with the demangled name.
"""
import argparse
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "damvsnet_amd", "csrc")


def table(unit, extra=()):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I" + os.path.join(REPO, "include"),
           "-I" + CSRC, "-x", "hip", "-c", os.path.join(CSRC, unit + ".hip"), "-o", os.devnull,
           "-Rpass-analysis=kernel-resource-usage"] + list(extra)
    err = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in err.splitlines():
        m = re.search(r"remark: (?:Function Name: (\S+)|\s*([A-Za-z /\[\]]+?): (\d+))", line)
        if not m:
            continue
        if m.group(1):
            cur = {"name": m.group(1)}
            rows.append(cur)
        elif cur is not None:
            cur[m.group(2).strip()] = int(m.group(3))
    names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                           text=True).stdout.splitlines()
    for r, n in zip(rows, names):
        r["name"] = re.sub(r"damvs::\(anonymous namespace\)::", "", n)
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("units", nargs="+")
    ap.add_argument("--grep", default="")
    a = ap.parse_args()
    for u in a.units:
        for r in table(u):
            if a.grep and not re.search(a.grep, r["name"]):
                continue
            print("%4d v %4d a  spill %3d  lds %6d  waves %d  %s" % (
                r.get("VGPRs", -1), r.get("AGPRs", -1), r.get("VGPRs Spill", -1), r.get("LDS Size [bytes/block]", -1),
                r.get("Occupancy [waves/SIMD]", -1), r["name"][:150]))


if __name__ == "__main__":
    sys.exit(main())
